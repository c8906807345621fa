"""Rebalanced frontier engine (ppls_amd/frontier.py) timing: one integral per run, sharded over the
ranks of `torch.distributed.run` (nccl = RCCL) or a single GPU. Prints one JSON line (rank 0).

  python tools/bench_frontier.py [--workload sin|cosh12|cosh10] [--reps 5] [--every 1]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/bench_frontier.py ...
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

WORK = {"sin": ("sin(1/x) on [1e-4, 1], EPSILON=1e-9 (BASELINE configs[3])", 1, 1e-4, 1.0, 1e-9, (56357, 28179)),
        "cosh12": ("cosh4 on [0, 5], EPSILON=1e-12 (BASELINE configs[4])", 0, 0.0, 5.0, 1e-12, (6606491, 3303246)),
        "cosh10": ("cosh4 on [0, 5], EPSILON=1e-10 (BASELINE configs[1])", 0, 0.0, 5.0, 1e-10, (1464273, 732137))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="sin", choices=sorted(WORK))
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--every", type=int, default=1)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    from ppls_amd import Context, Problem, frontier
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    desc, fid, a, b, eps, (tg, lg) = WORK[args.workload]
    p = Problem(fid, a, b, eps)
    with Context(local) as ctx:
        st = frontier.HipStepper(ctx)
        r = frontier.integrate(p, stepper=st, rebalance_every=args.every)   # warmup
        times = []
        for _ in range(args.reps):
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = frontier.integrate(p, stepper=st, rebalance_every=args.every)
            torch.cuda.synchronize()
            t = time.perf_counter() - t0
            if world > 1:
                tt = torch.tensor([t], dtype=torch.float64, device="cuda")
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                t = float(tt.item())
            times.append(t)
        ok = (r.tasks, r.accepted) == (tg, lg)
        # the static cyclic partition of the persistent engine, for the imbalance comparison
        per_shard = []
        if world == 1:
            for s in range(8):
                per_shard.append(ctx.integrate_shard(p, s, 8).tasks)
    if rank == 0:
        best = min(times)
        print(json.dumps({"engine": "frontier (level-synchronous, RCCL rebalance every %d level(s))" % args.every,
                          "workload": desc, "n_gpus": world, "verified": ok, "tasks": r.tasks,
                          "accepted": r.accepted, "levels": r.levels, "best_ms": best * 1e3,
                          "median_ms": sorted(times)[len(times) // 2] * 1e3,
                          "accepted_per_s": r.accepted / best, "rebalances": r.rebalances,
                          "moved_records": r.moved_records, "tasks_per_rank": r.tasks_per_rank,
                          "imbalance_rebalanced": max(r.tasks_per_rank) * world / r.tasks,
                          "static_cyclic_8_shards_tasks": per_shard,
                          "imbalance_static_cyclic_8": (max(per_shard) * 8 / sum(per_shard)) if per_shard else None}))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
