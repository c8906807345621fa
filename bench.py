#!/usr/bin/env python3
"""Benchmark: accepted subintervals/s (+ FP64 F-evals/s) for the reference integrand at EPSILON=1e-10.

Workload (BASELINE.json configs[1]): F(x)=cosh(x)^4 (aquadPartA.c:46) over [0,5] (:47-48) at
EPSILON=1e-10 -- 1 464 273 tasks, 732 137 accepted subintervals per integral. One step = one batch
of B (default 32768) such integrals through the hot path (persistent on-device farmer,
ppls_amd/csrc/aq_stream.h). With N ranks (one process per GPU, torch.distributed backend "nccl" =
RCCL) every integral is sharded: rank r evaluates shard r of N of each integral (the domain split
into subranges per GPU; strong scaling, total work fixed), and a rank packs up to N batches into
one persistent launch so a launch holds the same work whatever N. The partial results of the K
timed steps are combined with ONE all-reduce inside the timed region. Launches are pipelined
(no host sync between them); every integral's counts are verified bit-exactly against the golden
tree after timing.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--eps E] [--no-cpu-baseline]

Prints ONE JSON line (rank 0). `value` = accepted subintervals/s over all GPUs; roofline is the
persistent kernel's FP64 rate (38 algorithmic FLOP per task) over its HIP-event
launch time, against the 78.6 TFLOP/s FP64 vector peak of one MI355X; cpu_baseline is the
reference's bag of tasks restated on threads (oracle/aq_bag.c) timed on this host's cores.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FLOP_PER_TASK = 38          # exp 20 + cosh tail 3 + pow4 3 + step 12
FP64_PEAK = 78.6e12         # MI355X FP64 vector peak (256 CU x 2.4 GHz x 128 FLOP/clk), MI355X_MICROARCH.md
GOLDEN = {1e-10: (1464273, 732137), 1e-12: (6606491, 3303246), 1e-8: (319295, 159648), 1e-3: (6567, 3284)}


def host_cores():
    """CPU cores this process may use on this host, and the share it should load: the affinity set,
    capped by OMP_NUM_THREADS where the pool sets it (the GPU box: 16 cores per GPU)."""
    ncpu = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = ncpu
    try:
        share = min(ncpu, int(os.environ.get("OMP_NUM_THREADS", ncpu)))
    except ValueError:
        pass
    return ncpu, max(2, share)


def cpu_baseline(eps, target_s=12.0):
    """The reference's algorithm timed on this host's CPU cores (bounded sample), before any GPU init.

    SURVEY §8c/§8d: on the GPU host the CPU baseline is the build's own restatement of the farmer /
    worker bag of tasks (oracle/aq_bag.c: farmer + P-1 workers on threads, the reference's LIFO bag,
    dispatch loop and task body over the host libm), with P = the cores this process may load. Its
    totals must equal the reference's. (The reference binary itself is timed in the build container,
    BASELINE.md; it is not shipped here.) Falls back to the sequential oracle restatement."""
    tasks_golden, leaves_golden = GOLDEN.get(eps, (None, None))
    ncpu, nprocs = host_cores()
    bag = os.path.join(ROOT, "oracle", "_build", "aq_bag")
    if os.path.exists(bag) and leaves_golden and eps in (1e-3, 1e-10, 1e-12):
        try:
            runs, t_total = 0, 0.0
            while t_total < target_s and runs < 50:
                t0 = time.perf_counter()
                out = subprocess.run([bag, "-n", str(nprocs), "-e", repr(eps)], capture_output=True, text=True,
                                     timeout=120, check=True).stdout
                t_total += time.perf_counter() - t0
                runs += 1
                if sum(int(v) for v in out.strip().splitlines()[-1].split()) != tasks_golden:
                    raise RuntimeError("bag-of-tasks task total mismatch")
            return {"value": leaves_golden * runs / t_total, "unit": "accepted subintervals/s", "cores": nprocs,
                    "host_cpus": ncpu, "kind": "port",
                    "sample": f"{runs} full integrals (cosh4 [0,5], eps={eps}) by oracle/aq_bag -- the reference's "
                              f"farmer/worker bag of tasks on threads, farmer + {nprocs - 1} workers on {nprocs} of "
                              f"this host's {ncpu} CPUs -- {t_total:.1f} s wall; the single farmer thread "
                              f"(one message round trip per task, aquadPartA.c:145-171) bounds it, not the "
                              f"core count"}
        except Exception as e:
            print(f"cpu_baseline: oracle/aq_bag unusable ({e}); timing the sequential oracle", file=sys.stderr)
    from oracle import pyoracle as O
    runs, t_total, leaves = 0, 0.0, 0
    while t_total < target_s and runs < 400:
        t0 = time.perf_counter()
        r = O.integrate(eps=eps)
        t_total += time.perf_counter() - t0
        runs += 1
        leaves += r.leaves
    return {"value": leaves / t_total, "unit": "accepted subintervals/s", "cores": 1, "host_cpus": ncpu,
            "kind": "port", "sample": f"{runs} full integrals by the oracle's sequential restatement (1 thread), "
                                      f"{t_total:.1f} s"}


def load_traffic(tasks_per_launch):
    """HBM bytes per launch of the persistent kernel: the committed PMC profile's bytes per task
    (profiles/pmc_traffic.json, tools/profile_round.sh) times this launch's tasks (or None)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            per_task = json.load(f).get("hbm_bytes_per_task")
        return per_task * tasks_per_launch if per_task else None
    except Exception:
        return None


def ranks_seen(dist, coll, distributed):
    """How many ranks the process group really spans: an all-reduce of ones over it (RCCL under nccl),
    done before timing -- the line's n_gpus is checked against it, not just read from WORLD_SIZE."""
    if not distributed:
        return 1
    import torch
    one = torch.ones(1, dtype=torch.int64, device=coll)
    dist.all_reduce(one)
    return int(one.item())


def rank_stats(dist, coll, distributed, kern_ms, launches, tasks, elapsed):
    """Every rank's kernel time, launches and tasks over the timed region (one all-gather), and the
    imbalance max / mean of the kernel time and of the tasks (the farmer's per-worker counts, :162)."""
    import torch
    mine = torch.tensor([kern_ms, float(launches), float(tasks), elapsed], dtype=torch.float64, device=coll)
    if distributed:
        rows = [torch.zeros_like(mine) for _ in range(dist.get_world_size())]
        dist.all_gather(rows, mine)
    else:
        rows = [mine]
    rows = [r.cpu().tolist() for r in rows]
    ms = [r[0] for r in rows]
    tk = [int(r[2]) for r in rows]
    mean = lambda v: sum(v) / len(v) if v else 0.0
    return {"kernel_ms": ms, "launches": [int(r[1]) for r in rows], "tasks": tk, "elapsed_s": [r[3] for r in rows],
            "kernel_imbalance": max(ms) / mean(ms) if mean(ms) > 0 else None,
            "task_imbalance": max(tk) / mean(tk) if mean(tk) > 0 else None}


def bench_line(args, world, K, B, n_int, elapsed, accepted_total, f_evals, tot, per_launch, ctx_cus, single_ms,
               single_n, ok, backend, seen, stats, achieved, kern_avg_ms, tasks_per_launch, cpu, cu_stats=None):
    """The one JSON line rank 0 prints (the driver's contract plus roofline, cpu_baseline and the
    multi-rank fields: backend, ranks_seen -- counted by a collective -- and per-rank kernel time and
    tasks with their imbalance)."""
    return {
        "metric": "accepted subintervals/sec + FP64 F-evals/sec at 1/2/4/8 MI355X, EPSILON=1e-10",
        "value": accepted_total / elapsed,
        "unit": "accepted subintervals/s",
        "f_evals_per_sec": f_evals / elapsed,
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / K,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (analytic integrand, no dataset)",
        "config": {"workload": "cosh4 on [0,5], EPSILON=%g (BASELINE %s); one step = a batch of %d "
                               "such integrals, each sharded over the GPUs"
                               % (args.eps, {1e-10: "configs[1]", 1e-12: "configs[4]"}.get(args.eps, "off-config"), B),
                   "integrand": "cosh(x)^4 (aquadPartA.c:46)", "a": 0.0, "b": 5.0, "eps": args.eps,
                   "tasks_per_integral": int(tot[0, 1]), "accepted_per_integral": int(tot[0, 2]),
                   "parallelism": f"shard{world}" if world > 1 else "single-gpu",
                   "integrals_per_step": B,
                   "integrals_per_launch": per_launch,
                   "workgroups_per_gpu": ctx_cus},
        "single_integral_kernel_us": single_ms * 1e3 / single_n if single_n else None,
        "verified": ok,
        "backend": backend,
        "ranks_seen": seen,
        "per_rank": stats,
        "tasks_per_cu": cu_stats,
        "roofline": {"bound": "valu_fp64", "achieved": achieved / 1e12, "peak": FP64_PEAK / 1e12,
                     "unit": "TFLOP/s", "frac": achieved / FP64_PEAK, "traffic": load_traffic(tasks_per_launch),
                     "kernel": "aq::k_stream<0,false,false,false>", "kernel_avg_us": kern_avg_ms * 1e3,
                     "flop_per_task": FLOP_PER_TASK, "tasks_per_launch": tasks_per_launch},
        "cpu_baseline": cpu,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=8, help="timed batches")
    ap.add_argument("--warmup", type=int, default=2, help="untimed batches")
    ap.add_argument("--batch", type=int, default=32768,
                    help="integrals per step (one persistent launch per step on one GPU: ~0.5 ms of ramp-up and "
                         "end-of-launch tail per launch, 2 %% of an 8192-integral launch, 0.5 %% of 32768)")
    ap.add_argument("--eps", type=float, default=1e-10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-single", action="store_true",
                    help="skip the one-integral-per-launch latency probe (profiling runs: every dispatch is K-wide)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # launched by torch.distributed.run (even with one rank): a process group, so the combine below
    # runs through RCCL; a plain `python bench.py` is the single-GPU run with no group
    distributed = world > 1 or ("RANK" in os.environ and "MASTER_ADDR" in os.environ)
    if world != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)

    # CPU baseline first: before this process touches the GPU (child processes only).
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.eps)

    import numpy as np
    import torch
    import torch.distributed as dist
    from ppls_amd import Context, Problem

    # BENCH_SHARED_GPU=1 rehearses the N-rank path on a one-GPU box: every rank on device 0, the
    # collectives over gloo (RCCL needs one GPU per rank). Never set by the driver.
    shared = os.environ.get("BENCH_SHARED_GPU") == "1"
    dev = 0 if shared else local_rank
    torch.cuda.set_device(dev)
    if distributed:
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    coll = "cpu" if shared else "cuda"

    def all_reduce(t, op):
        if distributed:
            h = t.to(coll)
            dist.all_reduce(h, op=op)
            if h is not t:
                t.copy_(h)

    backend = dist.get_backend() if distributed else None
    seen = ranks_seen(dist, coll, distributed)
    if seen != world:
        print(f"bench: the process group spans {seen} ranks, WORLD_SIZE={world}", file=sys.stderr)

    ctx = Context(dev)
    ctx.set_level_histograms(False)
    problem = Problem(eps=args.eps)
    nslots = ctx.async_slots

    def barrier():
        if distributed:
            dist.barrier()

    B = args.batch
    if B < 1 or B > min(ctx.max_integrals_per_launch, nslots):
        raise SystemExit(f"--batch must be in [1, {min(ctx.max_integrals_per_launch, nslots)}]")
    # batches per launch: N of them (each rank holds 1/N of every integral), within the slot budget
    lb = max(1, min(world, min(ctx.max_integrals_per_launch, nslots) // B))

    def launch(m):
        # m integrals of the workload in one persistent launch (slots 0..m-1), this rank's shard
        if shared and world > 1:
            # rehearsal: persistent grids need the whole GPU, so the ranks sharing it take turns
            for r in range(world):
                if r == rank:
                    ctx.integrate_many_async(np.zeros(m), np.full(m, 5.0), args.eps, first_slot=0, shard=rank,
                                             nshards=world)
                    ctx.synchronize()
                dist.barrier()
            return
        ctx.integrate_many_async(np.zeros(m), np.full(m, 5.0), args.eps, first_slot=0, shard=rank, nshards=world)

    # single-integral latency (one integral per launch), reported beside the throughput: on one GPU
    # the kernel of the synchronous call a user makes for one integral (aq_integrate: its result slot
    # is re-zeroed by the fetch, so nothing is enqueued before the launch), on N the rank's shard
    single_ms, single_n = 0.0, 0
    if not args.no_single:
        from ppls_amd import Problem
        one = (lambda: ctx.integrate(Problem(eps=args.eps))) if world == 1 else (lambda: launch(1))
        one()                         # untimed: the first K=1 launch pays the K=1 setup
        ctx.synchronize()
        ctx.kernel_timing(True)
        for _ in range(max(args.warmup, 5)):
            one()
        ctx.synchronize()
        single_ms, single_n = ctx.kernel_time()
        ctx.kernel_timing(False)

    # warmup (also validates)
    w = 0
    while w < max(1, args.warmup):
        m = min(max(1, args.warmup) - w, lb)
        launch(m * B)
        w += m
    ctx.synchronize()

    ctx.cu_task_counters(reset=True)   # per-CU task counters over the timed launches only
    K = args.steps
    n_int = K * B
    totals = torch.zeros((n_int, 4), dtype=torch.float64, device="cuda")
    ctx.kernel_timing(True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    done = 0
    while done < K:
        # launches queue back to back on the context's stream: each gathers its slots' results into
        # its rows of `totals` (device memory), and the next launch re-zeroes the slots after that
        m = min(K - done, lb)
        launch(m * B)
        ctx.gather_results(0, m * B, totals.data_ptr() + done * B * 4 * totals.element_size())
        done += m
    ctx.synchronize()
    my_tasks = totals[:, 1].sum()           # this rank's tasks (its shards), before the combine
    all_reduce(totals, dist.ReduceOp.SUM)   # shard partials -> whole integrals
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    kern_ms, launches = ctx.kernel_time()
    ctx.kernel_timing(False)

    elapsed = t1 - t0
    stats = rank_stats(dist, coll if distributed else "cpu", distributed, kern_ms, launches, float(my_tasks.item()),
                       elapsed)
    if distributed:
        tt = torch.tensor([elapsed, kern_ms / max(launches, 1)], dtype=torch.float64, device="cuda")
        all_reduce(tt, dist.ReduceOp.MAX)
        elapsed, kern_avg_ms = float(tt[0]), float(tt[1])
    else:
        kern_avg_ms = kern_ms / max(launches, 1)
    per_launch = n_int / max(launches, 1)

    # this rank's tasks per CU over the timed launches (every launch shape keeps them: aq_cu_task_counters)
    cu = ctx.cu_task_counters(reset=True)
    cu_v = list(cu.values())
    cu_stats = {"n_cu": len(cu_v), "min": min(cu_v) if cu_v else 0, "max": max(cu_v) if cu_v else 0,
                "imbalance": (max(cu_v) * len(cu_v) / sum(cu_v)) if cu_v and sum(cu_v) else None,
                "sum": sum(cu_v)}

    # verify every timed step against the golden tree
    tot = totals.cpu().numpy()
    tg, lg = GOLDEN.get(args.eps, (None, None))
    ok = bool((tot[:, 3] == 0).all()) and seen == world and cu_stats["sum"] == int(my_tasks.item())
    if tg is not None:
        ok = ok and bool((tot[:, 1] == tg).all() and (tot[:, 2] == lg).all())
    accepted_total = float(tot[:, 2].sum())
    tasks_total = float(tot[:, 1].sum())
    f_evals = tasks_total + 2 * n_int   # algorithmic F evaluations: 1 per task + F(A), F(B) per integral

    # this rank's share of the tasks per launch, for the roofline of its kernel
    mine = ctx.fetch(0)
    tasks_per_launch = mine.tasks * per_launch
    achieved = FLOP_PER_TASK * tasks_per_launch / (kern_avg_ms * 1e-3) if kern_avg_ms > 0 else 0.0

    if rank == 0:
        out = bench_line(args, world, K, B, n_int, elapsed, accepted_total, f_evals, tot, per_launch, ctx.num_cus,
                         single_ms, single_n, ok, backend, seen, stats, achieved, kern_avg_ms, tasks_per_launch, cpu,
                         cu_stats)
        print(json.dumps(out))
    ctx.close()
    if distributed:
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
