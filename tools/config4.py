"""Config 4 of BASELINE.json (sin(1/x) on [1e-4, 1], EPSILON=1e-9, "sharded over 8 GPUs, heavy load
imbalance, RCCL rebalance") measured on ONE GPU (diagnostic tool; DESIGN.md §6 records the decision).

  python tools/config4.py lone [--reps 20]
      one integral: k_stream (aq_integrate-shaped launch, kernel time by HIP events) against
      ppls_amd.frontier.integrate (the level-synchronous engine: one launch + one host sync per
      level; wall time), both on this process alone.

  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P \\
      tools/config4.py batch [--integrals 4096] [--shards S]
      a batch of M sin(1/x) integrals over N ranks that share cuda:0 (gloo collectives; the ranks take
      turns on the GPU, since a persistent grid needs all of it) through
      dist.integrate_batch_distributed, static partition (shard s of every integral on rank s mod N)
      against the rebalanced one (LPT over measured shard costs, between launches). Each rank's kernel
      time is its own launches only, so max over ranks = the makespan N real GPUs would see.

Prints one JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

A, B, EPS = 1e-4, 1.0, 1e-9


def golden():
    t = json.load(open(os.path.join(ROOT, "tests", "golden", "trees.json")))["sin_recip_eps1e-9"]
    return t["tasks"], t["leaves"]


def lone(args):
    import torch
    from ppls_amd import Context, Problem, SIN_RECIP, frontier
    g_tasks, g_leaves = golden()
    ctx = Context(0)
    ctx.set_level_histograms(False)
    p = Problem(integrand=SIN_RECIP, a=A, b=B, eps=EPS)
    ctx.integrate_async(p, 0)
    ctx.synchronize()
    ctx.kernel_timing(True)
    for _ in range(args.reps):
        ctx.integrate_async(p, 0)
    ms, n = ctx.kernel_time()
    ctx.kernel_timing(False)
    r = ctx.fetch(0)
    out = {"lone_k_stream_kernel_us": ms * 1e3 / n, "k_stream_counts_ok": (r.tasks, r.accepted) == (g_tasks, g_leaves)}
    t0 = time.perf_counter()
    r = ctx.integrate(p)
    out["lone_k_stream_wall_us"] = (time.perf_counter() - t0) * 1e6
    stepper = frontier.HipStepper(ctx)
    fr = frontier.integrate(p, stepper=stepper)         # warm-up (buffers, first launches)
    t0 = time.perf_counter()
    reps = 5
    for _ in range(reps):
        fr = frontier.integrate(p, stepper=stepper)
    torch.cuda.synchronize()
    out["lone_frontier_wall_us"] = (time.perf_counter() - t0) * 1e6 / reps
    out["frontier_counts_ok"] = (fr.tasks, fr.accepted) == (g_tasks, g_leaves)
    out["frontier_levels"] = fr.levels
    out["tasks"] = g_tasks
    print(json.dumps(out))
    ctx.close()


class TurnRunner:
    """HipBatchRunner for ranks that share one GPU: in every round the ranks launch one after
    another (barriers), so each rank's kernel time is its own launch alone."""

    def __init__(self, ctx, rank, world):
        from ppls_amd.dist import HipBatchRunner
        self.inner = HipBatchRunner(ctx)
        self.rank, self.world, self.ms = rank, world, 0.0

    def run(self, a, b, shards, nshards, eps, integrand):
        import torch.distributed as dist
        from ppls_amd.dist import ROW
        rows = np.zeros((0, ROW), np.int64)
        for r in range(self.world):
            if r == self.rank:
                rows = self.inner.run(a, b, shards, nshards, eps, integrand)
                self.ms = getattr(self.inner, "ms", 0.0) if len(a) else 0.0
            dist.barrier()
        return rows


def batch(args):
    import torch
    import torch.distributed as dist
    from ppls_amd import Context, SIN_RECIP
    from ppls_amd.dist import integrate_batch_distributed
    g_tasks, g_leaves = golden()
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    ctx = Context(0)
    ctx.set_level_histograms(False)
    m = args.integrals
    a, b = np.full(m, A), np.full(m, B)
    runner = TurnRunner(ctx, rank, world)
    out = {"m": m, "world": world, "tasks_per_integral": g_tasks}
    for name, reb in (("static", False), ("rebalanced", True)):
        integrate_batch_distributed(a[:64], b[:64], EPS, SIN_RECIP, runner=runner, shards_per_integral=args.shards,
                                    rebalance=reb)                     # warm-up
        t0 = time.perf_counter()
        res = integrate_batch_distributed(a, b, EPS, SIN_RECIP, runner=runner, shards_per_integral=args.shards,
                                          rebalance=reb)
        wall = time.perf_counter() - t0
        ms = res.kernel_ms_per_rank
        out[name] = {"counts_ok": bool((res.tasks == g_tasks).all() and (res.accepted == g_leaves).all()),
                     "rounds": res.rounds, "tasks_per_rank": res.tasks_per_rank,
                     "task_imbalance": max(res.tasks_per_rank) / (sum(res.tasks_per_rank) / world),
                     "kernel_ms_per_rank": [round(x, 3) for x in ms],
                     "makespan_ms": max(ms), "ideal_ms": sum(ms) / world,
                     "predicted_imbalance_last": res.predicted_imbalance[-1],
                     "wall_s_shared_gpu": wall}
    if rank == 0:
        print(json.dumps(out))
    ctx.close()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["lone", "batch"])
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--integrals", type=int, default=4096)
    ap.add_argument("--shards", type=int, default=None, help="shards per integral (default 4 x ranks)")
    args = ap.parse_args()
    lone(args) if args.mode == "lone" else batch(args)


if __name__ == "__main__":
    main()
