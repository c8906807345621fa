#!/usr/bin/env python3
"""Benchmark: accepted subintervals/s (+ FP64 F-evals/s) for the reference integrand at EPSILON=1e-10.

Workload (BASELINE.json configs[1]): F(x)=cosh(x)^4 (aquadPartA.c:46) over [0,5] (:47-48) at
EPSILON=1e-10 -- 1 464 273 tasks, 732 137 accepted subintervals per integral. One step = one batch
of B (default 32768) such integrals through the hot path (persistent on-device farmer,
ppls_amd/csrc/aq_stream.h). With N ranks (one process per GPU, torch.distributed backend "nccl" =
RCCL) every integral is sharded: each rank evaluates one shard of N of each integral (the domain
split into subranges per GPU; strong scaling, total work fixed) -- rank r shard (r + i) mod N of the
launch's i-th integral, so every rank gets every shard equally often and the snake partition's
per-shard skew (1.5 % at 8 shards) cancels -- and a rank packs N batches into one persistent launch
(a launch holds up to 262144 integrals: N x 32768 shards of 1/N each, the work of one GPU's
32768-integral launch, whatever N <= 8). The partial results of the K timed steps are combined with
ONE all-reduce inside the timed region. Launches are pipelined
(no host sync between them); every integral's counts are verified bit-exactly and its area to
1e-12 relative against the golden tree after timing.

After the headline's timed region, four secondary passes are timed the same way (barrier + sync on
both sides, max over ranks) and reported under "secondary":
  * C3 (BASELINE configs[2]): 1 000 000 splitmix64-bounded integrals at EPSILON=1e-10, split into
    contiguous whole-integral blocks per rank, through the batch front end (aq_integrate_batch);
    verified by T = 2L - 1 for every integral, the committed per-integral prefix and the exact KAT
    (Σ leaves of the first 10 000 draws, tests/golden/batch.json);
  * C5 (BASELINE configs[4]): EPSILON=1e-12, 4096 copies of the integral per pass, each sharded over
    the N GPUs; verified against the golden tree (counts exact, area to 1e-12);
  * C4 (BASELINE configs[3]): sin(1/x) on [1e-4, 1] at EPSILON=1e-9, 4096 copies per pass as whole
    integrals in contiguous blocks per rank, and the lone integral's kernel time; verified against the
    golden sin(1/x) tree;
  * C3 again at EPSILON=1e-3 (SURVEY §8d's launch/compaction-bound run: ~1 400 tasks per integral),
    verified the same way (the first 256 integrals, the 10 000-draw KAT: mean leaves 711.4936).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--eps E] [--no-cpu-baseline]

--gpus N > 1 with no launcher (WORLD_SIZE unset): this process times the CPU baseline first (no GPU
call), then runs N ranks itself through `torch.distributed.run` and exits with their status. Under a
launcher WORLD_SIZE must equal --gpus (aquadPartA.c:86-90: the process count is the launch's, and a
mismatch is an error, not a fallback).

Prints ONE JSON line (rank 0). `value` = accepted subintervals/s over all GPUs; roofline is the
persistent kernel's FP64 rate (38 algorithmic FLOP per task) over its HIP-event
launch time, against the 78.6 TFLOP/s FP64 vector peak of one MI355X; cpu_baseline is the
reference's bag of tasks restated on threads (oracle/aq_bag.c) timed on this host's cores.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FLOP_PER_TASK = 38          # exp 20 + cosh tail 3 + pow4 3 + step 12
FP64_PEAK = 78.6e12         # MI355X FP64 vector peak (256 CU x 2.4 GHz x 128 FLOP/clk), MI355X_MICROARCH.md
# eps -> (tasks, accepted, quad-precision Σ of the leaf areas) of cosh4 on [0,5] (tests/golden/trees.json,
# pinned by the reference binary's own runs)
GOLDEN = {1e-10: (1464273, 732137, 7583461.361505481304452902),
          1e-12: (6606491, 3303246, 7583461.361497082882355142),
          1e-8: (319295, 159648, 7583461.361685127681076307),
          1e-3: (6567, 3284, 7583461.801486495444390989)}
AREA_RTOL = 1e-12           # the north star's area tolerance
C3_N = 1_000_000
C5_COPIES = 4096
C4_COPIES = 4096
C4 = (1e-4, 1.0, 1e-9)      # BASELINE configs[3]: sin(1/x) on [1e-4, 1] at EPSILON=1e-9
SPLITMIX_GOLDEN = 0x9E3779B97F4A7C15
CPU_ENV = "BENCH_CPU_BASELINE"   # the launcher's CPU baseline, handed to rank 0 (JSON)


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
    tasks_golden, leaves_golden = GOLDEN.get(eps, (None, None, None))[:2]
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


def load_json(rel):
    try:
        with open(os.path.join(ROOT, rel)) as f:
            return json.load(f)
    except Exception:
        return None


def load_traffic(tasks_per_launch):
    """HBM bytes per launch of the persistent kernel: the committed PMC profile's bytes per task
    (profiles/pmc_traffic.json, tools/profile_round.sh) times this launch's tasks (or None). Not
    measured in this run: PMC counters need their own profiler passes."""
    per_task = (load_json(os.path.join("profiles", "pmc_traffic.json")) or {}).get("hbm_bytes_per_task")
    return per_task * tasks_per_launch if per_task else None


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


def areas_ok(areas, want):
    """Every area within AREA_RTOL (relative) of the golden quad Σ."""
    import numpy as np
    return bool(np.all(np.abs(np.asarray(areas, np.float64) - want) <= AREA_RTOL * abs(want)))


def splitmix64_bounds(n):
    """state += golden; standard mix; u = (z >> 11) * 2^-53; a = 5u1, b = 5u2, swap."""
    import numpy as np
    with np.errstate(over="ignore"):
        k = np.arange(1, 2 * n + 1, dtype=np.uint64)
        z = np.uint64(SPLITMIX_GOLDEN) + k * np.uint64(SPLITMIX_GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
    a, b = 5.0 * u[0::2], 5.0 * u[1::2]
    return np.minimum(a, b), np.maximum(a, b)


def ubench_step2():
    """The two-pairs-per-lane microbenchmark of the kernel's per-pair arithmetic (profiles/ceiling.json,
    tools/ubench_step2.hip), or None. It is NOT a bound on the kernel: its loop issues 76 FP64 + 33
    other VALU per pair against the round's 76 + 22 -- a reference figure only."""
    return load_json(os.path.join("profiles", "ceiling.json"))


def issue_bound():
    """The kernel's own VALU-issue bound from its committed rocprofv3 counters (profiles/pmc_valu.json,
    tools/r05_pmc_valu.sh + tools/pmc_valu.py on this launch shape): the algorithmic frac the measured
    instruction stream would reach with the SIMD's VALU issuing every cycle, frac / VALU busy, with
    VALU busy = 3 waves/SIMD x SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES. None when absent."""
    return load_json(os.path.join("profiles", "pmc_valu.json"))


def launch_plan(steps, per_launch):
    """Steps per persistent launch for K timed steps: per_launch (N at N ranks: each rank packs N
    batches of 1/N shards into one launch) each, the remainder last -- K = 20 at N = 8 is 8 + 8 + 4."""
    plan, done = [], 0
    while done < steps:
        m = min(steps - done, per_launch)
        plan.append(m)
        done += m
    return plan


def shard_rotation(rank, world, m):
    """The shard of each of a launch's m integrals on this rank: (rank + i) mod N, so every rank
    evaluates every shard of the snake partition equally often whenever m is a multiple of N (its
    per-shard skew, 1.5 % at 8 shards, cancels instead of landing on one rank)."""
    import numpy as np
    return (rank + np.arange(m)) % world


def agree_on_workers(dist, coll, distributed, num_workers):
    """Every rank's persistent worker count (waves per launch) must be the same: the shard partition
    (shares, seed depth) is a function of it, and ranks on different partitions would combine shards
    of different trees into wrong counts with no error (AQ_GRID, CU counts). One all-gather
    before the first sharded launch; a mismatch is an error exit on every rank."""
    if not distributed:
        return [num_workers]
    import torch
    mine = torch.tensor([num_workers], dtype=torch.int64, device=coll)
    rows = [torch.zeros_like(mine) for _ in range(dist.get_world_size())]
    dist.all_gather(rows, mine)
    seen = [int(r.item()) for r in rows]
    if len(set(seen)) != 1:
        raise SystemExit(f"bench: ranks disagree on the persistent worker count {seen} (AQ_GRID / CU count): "
                         f"their shard partitions would differ")
    return seen


def bench_line(args, world, K, B, n_int, elapsed, accepted_total, f_evals, tot, per_launch, ctx_cus, single_ms,
               single_n, ok, backend, seen, stats, achieved, kern_avg_ms, tasks_per_launch, cpu, cu_stats=None,
               secondary=None, checks=None):
    """The one JSON line rank 0 prints (the driver's contract plus roofline, cpu_baseline and the
    multi-rank fields: backend, ranks_seen -- counted by a collective -- and per-rank kernel time and
    tasks with their imbalance)."""
    ub = ubench_step2() or {}
    ib = issue_bound() or {}
    ibd = ib.get("derived", {})
    frac = achieved / FP64_PEAK
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
                   # a launch of m shards of 1/N of an integral each holds m / N integrals' work
                   "integral_equivalents_per_launch": per_launch / world,
                   "workgroups_per_gpu": ctx_cus[0], "waves_per_gpu": ctx_cus[1], "cus_per_gpu": ctx_cus[2]},
        "single_integral_kernel_us": single_ms * 1e3 / single_n if single_n else None,
        "verified": ok,
        "checks": checks,
        "backend": backend,
        "ranks_seen": seen,
        "per_rank": stats,
        "tasks_per_cu": cu_stats,
        "roofline": {"bound": "valu_fp64", "achieved": achieved / 1e12, "peak": FP64_PEAK / 1e12,
                     "unit": "TFLOP/s", "frac": frac, "traffic": load_traffic(tasks_per_launch),
                     "traffic_source": "not measured in this run: profiles/pmc_traffic.json's PMC bytes per task "
                                       "(FETCH_SIZE x2 + WRITE_SIZE passes) x this launch's tasks",
                     # the kernel's own VALU-issue bound (measured counters of this launch shape, committed)
                     "issue_bound": ibd.get("issue_bound_frac"),
                     "frac_of_issue_bound": frac / ibd["issue_bound_frac"] if ibd.get("issue_bound_frac") else None,
                     "valu_busy": ibd.get("valu_busy"),
                     "fp64_hw_frac": ibd.get("frac_fp64_hw"),
                     "issue_bound_source": "profiles/pmc_valu.json (%s): frac / VALU busy of the committed rocprofv3 "
                                           "SQ counters, VALU busy = 3 x SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES; "
                                           "fp64_hw_frac = 64 x (ADD + MUL + TRANS + 2 FMA) F64 wave-instructions "
                                           "per second / peak (idle lanes included)" % ib.get("tag", "?"),
                     "ubench_step2_frac": ub.get("frac"),
                     "ubench_step2_note": "two independent pairs per lane of the per-pair arithmetic "
                                          "(tools/ubench_step2.hip); 76 FP64 + 33 other VALU per pair against the "
                                          "round's 76 + 22 -- a reference figure, not a bound on the kernel",
                     "kernel": "aq::k_stream<0,false,false,false,12,false>", "kernel_avg_us": kern_avg_ms * 1e3,
                     "flop_per_task": FLOP_PER_TASK, "tasks_per_launch": tasks_per_launch},
        "cpu_baseline": cpu,
        "secondary": secondary,
    }


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launcher_cmd(n, argv, port):
    """One rank per GPU of this node (the driver's own launch line)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def spawn_ranks(args, argv, runner=None, baseline=cpu_baseline):
    """--gpus N > 1 without a launcher: time the CPU baseline here (this process makes no GPU call),
    run N ranks as a child `torch.distributed.run`, hand the baseline to rank 0 through the
    environment, and return the children's exit status (non-zero if any rank failed)."""
    env = dict(os.environ)
    # RCCL's intra-node transport and torch's CUDA-tensor sharing use HIP IPC handles; this host
    # driver supports only the dmabuf IPC mode, and without HSA_ENABLE_IPC_MODE_LEGACY=0 every
    # cross-process handle fails (`hipIpcGetMemHandle: invalid argument`). The GPU pool exports it;
    # the ranks get it explicitly, before any GPU call, whatever the parent's environment
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if not args.no_cpu_baseline:
        env[CPU_ENV] = json.dumps(baseline(args.eps))
    runner = runner or (lambda cmd, env: subprocess.call(cmd, env=env))
    return runner(launcher_cmd(args.gpus, argv, free_port()), env)


def parse(argv):
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
    ap.add_argument("--no-secondary", action="store_true", help="skip the C3 / C5 passes after the headline")
    ap.add_argument("--c3-n", type=int, default=C3_N, help="integrals of the C3 pass")
    return ap.parse_args(argv)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args, argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        sys.exit(2)
    # launched by torch.distributed.run (even with one rank): a process group, so the combine below
    # runs through RCCL; a plain `python bench.py` is the single-GPU run with no group
    distributed = world > 1 or ("RANK" in os.environ and "MASTER_ADDR" in os.environ)

    # CPU baseline first: before this process touches the GPU (child processes only). Handed over by
    # this script's own launcher, else timed by rank 0 here (the other ranks wait in the rendezvous).
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = json.loads(os.environ[CPU_ENV]) if os.environ.get(CPU_ENV) else cpu_baseline(args.eps)

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

    def reduce_list(vals, op):
        t = torch.tensor(vals, dtype=torch.float64, device="cuda")
        all_reduce(t, op)
        return t.cpu().tolist()

    backend = dist.get_backend() if distributed else None
    seen = ranks_seen(dist, coll, distributed)
    if seen != world:
        print(f"bench: the process group spans {seen} ranks, WORLD_SIZE={world}", file=sys.stderr)

    ctx = Context(dev)
    ctx.set_level_histograms(False)
    nslots = ctx.async_slots
    agree_on_workers(dist, coll, distributed, ctx.num_workers)

    def barrier():
        if distributed:
            dist.barrier()

    def in_turn(fn):
        """Run fn on this rank; in the shared-GPU rehearsal the ranks take turns (persistent grids
        need the whole GPU), each finishing before the next starts."""
        if shared and world > 1:
            out = None
            for r in range(world):
                if r == rank:
                    out = fn()
                    ctx.synchronize()
                dist.barrier()
            return out
        return fn()

    B = args.batch
    cap = min(ctx.max_integrals_per_launch, nslots)
    if B < 1 or B > cap:
        raise SystemExit(f"--batch must be in [1, {cap}]")
    # batches per launch: N of them (each rank holds 1/N of every integral), within the slot budget
    lb = max(1, min(world, cap // B))

    def launch(m, eps=args.eps):
        # m integrals of the workload in one persistent launch (slots 0..m-1), this rank's shards: the
        # i-th integral's shard (rank + i) mod N (every rank holds each shard of 1/N of the integrals)
        if world == 1:
            in_turn(lambda: ctx.integrate_many_async(np.zeros(m), np.full(m, 5.0), eps, first_slot=0))
        else:
            sh = shard_rotation(rank, world, m)
            in_turn(lambda: ctx.integrate_mixed_async(np.zeros(m), np.full(m, 5.0), sh, world, eps, first_slot=0))

    # single-integral latency (one integral per launch), reported beside the throughput: on one GPU
    # the kernel of the synchronous call a user makes for one integral (aq_integrate: its result slot
    # is re-zeroed by the fetch, so nothing is enqueued before the launch), on N the rank's shard
    single_ms, single_n = 0.0, 0
    if not args.no_single:
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
    for m in launch_plan(max(1, args.warmup), lb):
        launch(m * B)
    ctx.synchronize()

    ctx.cu_task_counters(reset=True)   # per-CU task counters over the timed launches only
    K = args.steps
    n_int = K * B
    totals = torch.zeros((n_int, 4), dtype=torch.float64, device="cuda")
    # torch loads a kernel's code object at its first use: the column sum below (bookkeeping, not the
    # hot path) had paid a ~25 ms one-time load inside the timed region -- 1.2 ms of every step's
    # ms_per_step at 20 steps (rocprofv3 kernel trace, profiles/r06a: a 25.7 ms gap before the first
    # reduce_kernel). Loaded here, untimed.
    float(totals[:, 1].sum().item())
    ctx.kernel_timing(True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    done = 0
    for m in launch_plan(K, lb):
        # launches queue back to back on the context's stream: each gathers its slots' results into
        # its rows of `totals` (device memory), and the next launch re-zeroes the slots after that
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
        elapsed, kern_avg_ms = reduce_list([elapsed, kern_ms / max(launches, 1)], dist.ReduceOp.MAX)
    else:
        kern_avg_ms = kern_ms / max(launches, 1)
    per_launch = n_int / max(launches, 1)

    # this rank's tasks per CU over the timed launches (every launch shape keeps them: aq_cu_task_counters)
    cu = ctx.cu_task_counters(reset=True)
    cu_v = list(cu.values())
    cu_stats = {"n_cu": len(cu_v), "min": min(cu_v) if cu_v else 0, "max": max(cu_v) if cu_v else 0,
                "imbalance": (max(cu_v) * len(cu_v) / sum(cu_v)) if cu_v and sum(cu_v) else None,
                "sum": sum(cu_v)}

    # verify every timed step against the golden tree: counts exact, areas to AREA_RTOL
    tot = totals.cpu().numpy()
    tg, lg, ag = GOLDEN.get(args.eps, (None, None, None))
    checks = {"errors": bool((tot[:, 3] == 0).all()), "ranks": seen == world,
              "cu_counters": cu_stats["sum"] == int(my_tasks.item())}
    if tg is not None:
        checks["counts"] = bool((tot[:, 1] == tg).all() and (tot[:, 2] == lg).all())
        checks["areas"] = areas_ok(tot[:, 0], ag)
    # every rank's view (the per-CU check is per rank)
    checks = dict(zip(checks, (bool(v) for v in reduce_list([float(v) for v in checks.values()], dist.ReduceOp.MIN))))
    ok = all(checks.values())
    accepted_total = float(tot[:, 2].sum())
    tasks_total = float(tot[:, 1].sum())
    f_evals = tasks_total + 2 * n_int   # algorithmic F evaluations: 1 per task + F(A), F(B) per integral

    # this rank's tasks per launch (its shards), for the roofline of its kernel
    tasks_per_launch = float(my_tasks.item()) / max(launches, 1)
    achieved = FLOP_PER_TASK * tasks_per_launch / (kern_avg_ms * 1e-3) if kern_avg_ms > 0 else 0.0

    secondary = None
    if not args.no_secondary:
        secondary = [
            c3_pass(ctx, args, rank, world, barrier, in_turn, reduce_list, dist),
            c5_pass(ctx, rank, world, barrier, launch, reduce_list, dist, torch, all_reduce),
            c4_pass(ctx, rank, world, barrier, in_turn, reduce_list, dist, torch),
            c3_pass(ctx, args, rank, world, barrier, in_turn, reduce_list, dist, eps=1e-3),
        ]
        ok = ok and all(s["verified"] for s in secondary)

    if rank == 0:
        # the persistent launch's shape behind the roofline: workgroups (waves / 12: 768-thread
        # workgroups), waves and the device's CUs (AQ_GRID can set fewer workgroups than CUs)
        shape = (ctx.num_workers // 12, ctx.num_workers, ctx.num_cus)
        out = bench_line(args, world, K, B, n_int, elapsed, accepted_total, f_evals, tot, per_launch, shape,
                         single_ms, single_n, ok, backend, seen, stats, achieved, kern_avg_ms, tasks_per_launch, cpu,
                         cu_stats, secondary, checks)
        print(json.dumps(out))
    ctx.close()
    if distributed:
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


# tests/golden/batch.json keys per C3 tolerance: per-integral leaves and areas of a prefix, and the
# exact Σ of the KAT prefix (mean leaves 711.5 at 1e-3, 153 330.8 at 1e-10)
C3_GOLDEN = {
    1e-10: {"leaves": "leaves_eps1e-10", "area_hex": "area_eps1e-10_hex", "kat_n": "kat_n_eps1e-10",
            "kat_leaves": "kat_sum_leaves_eps1e-10", "kat_tasks": "kat_sum_tasks_eps1e-10"},
    1e-3: {"leaves": "leaves_eps1e-3_first256", "area_hex": "area_eps1e-3_first256_hex", "kat_n": "n_eps1e-3",
           "kat_leaves": "sum_leaves_eps1e-3", "kat_tasks": "sum_tasks_eps1e-3"},
}


def c3_pass(ctx, args, rank, world, barrier, in_turn, reduce_list, dist, eps=1e-10):
    """BASELINE configs[2]: 1 M splitmix64-bounded integrals at EPSILON=1e-10 (the throughput run) or
    1e-3 (tiny trees: launch- and seeding-bound), contiguous whole-integral blocks per rank through
    aq_integrate_batch (up to 262144 integrals per persistent launch)."""
    import numpy as np
    import torch
    keys = C3_GOLDEN[eps]
    n = args.c3_n
    a, b = splitmix64_bounds(n)
    lo, hi = rank * n // world, (rank + 1) * n // world
    # untimed: one launch of this workload sizes the jobs of the next (the launch-to-launch hint)
    w = min(hi - lo, 65536)
    in_turn(lambda: ctx.integrate_batch(a[lo:lo + w], b[lo:lo + w], eps))
    ctx.kernel_timing(True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    area, tasks, acc = in_turn(lambda: ctx.integrate_batch(a[lo:hi], b[lo:hi], eps))
    barrier()
    t1 = time.perf_counter()
    kern_ms, launches = ctx.kernel_time()
    ctx.kernel_timing(False)
    ok = bool((tasks == 2 * acc - 1).all())
    golden = load_json(os.path.join("tests", "golden", "batch.json")) or {}
    checked = []
    if lo == 0:
        pre = golden.get(keys["leaves"]) or []
        m = min(len(pre), hi)
        if m:
            ok = ok and bool((acc[:m] == np.asarray(pre[:m], np.uint64)).all())
            want = np.array([float.fromhex(v) for v in golden[keys["area_hex"]][:m]])
            ok = ok and bool(np.all(np.abs(area[:m] - want) <= AREA_RTOL * np.abs(want)))
            checked.append(f"counts and areas of integrals 0..{m - 1} vs tests/golden/batch.json")
        kn = golden.get(keys["kat_n"], 0)
        if kn and hi >= kn:
            ok = ok and int(acc[:kn].sum()) == golden[keys["kat_leaves"]] \
                and int(tasks[:kn].sum()) == golden[keys["kat_tasks"]]
            checked.append(f"exact Σ leaves / tasks of the first {kn} draws (mean leaves "
                           f"{golden[keys['kat_leaves']] / kn:.4f})")
    # every rank's accepted / tasks / kernel seconds / verdict summed, the wall time's max
    leaves, tsum, ksum, okall = reduce_list([float(acc.sum()), float(tasks.sum()), kern_ms / 1e3, 1.0 if ok else 0.0],
                                            dist.ReduceOp.SUM)
    elapsed, = reduce_list([t1 - t0], dist.ReduceOp.MAX)
    return {"workload": "C3 (BASELINE configs[2]): %d splitmix64-bounded cosh4 integrals at EPSILON=%g, "
                        "whole integrals in contiguous blocks per rank" % (n, eps),
            "value": leaves / elapsed, "unit": "accepted subintervals/s", "ms": elapsed * 1e3,
            "integrals_per_s": n / elapsed, "accepted": int(leaves), "tasks": int(tsum),
            "frac": FLOP_PER_TASK * tsum / ksum / FP64_PEAK if ksum > 0 else None,
            "verified": okall == world, "checks": ["T = 2L - 1 for every integral"] + checked}


def c4_pass(ctx, rank, world, barrier, in_turn, reduce_list, dist, torch):
    """BASELINE configs[3]: sin(1/x) on [1e-4, 1] at EPSILON=1e-9 (the skewed tree: nearly all of its
    56 357 tasks lie in one small region near 1e-4). C4_COPIES copies per pass as WHOLE integrals in
    contiguous blocks per rank -- its per-integral shards are seeding-bound, whole trees are not
    (a batch of config-4 integrals is distributed as whole integrals) -- one untimed launch
    that sizes the jobs, two timed; and the lone integral's kernel time (the synchronous call, 8
    launches). Verified: every copy's counts exact and area within 1e-12 of the golden tree's quad Σ
    (tests/golden/trees.json, pinned by the reference binary built with that F)."""
    import numpy as np
    from ppls_amd import Problem, SIN_RECIP
    a0, b0, eps = C4
    g = (load_json(os.path.join("tests", "golden", "trees.json")) or {}).get("sin_recip_eps1e-9") or {}
    m = C4_COPIES
    lo, hi = rank * m // world, (rank + 1) * m // world
    mine = hi - lo
    A, B = np.full(mine, a0), np.full(mine, b0)

    def run():
        ctx.integrate_many_async(A, B, eps, first_slot=0, integrand=SIN_RECIP)

    in_turn(run)                        # untimed: sizes the jobs (the launch-to-launch hint)
    ctx.synchronize()
    reps = 2
    rows = torch.zeros((reps * max(mine, 1), 4), dtype=torch.float64, device="cuda")
    ctx.kernel_timing(True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(reps):
        in_turn(run)
        ctx.gather_results(0, mine, rows.data_ptr() + i * mine * 4 * rows.element_size())
    ctx.synchronize()
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    kern_ms, launches = ctx.kernel_time()
    ctx.kernel_timing(False)
    tot = rows.cpu().numpy()[:reps * mine]
    ok = bool(g) and bool((tot[:, 3] == 0).all() and (tot[:, 1] == g["tasks"]).all() and
                          (tot[:, 2] == g["leaves"]).all()) and areas_ok(tot[:, 0], float(g["area_quad"]))
    # the lone integral (one launch per integral, on every rank)
    p = Problem(SIN_RECIP, a0, b0, eps)
    ctx.integrate(p)
    ctx.kernel_timing(True)
    for _ in range(8):
        r = ctx.integrate(p)
    lone_ms, lone_n = ctx.kernel_time()
    ctx.kernel_timing(False)
    ok = ok and bool(g) and (r.tasks, r.accepted) == (g["tasks"], g["leaves"])
    elapsed, lone_us = reduce_list([t1 - t0, lone_ms * 1e3 / max(lone_n, 1)], dist.ReduceOp.MAX)
    leaves, tasks, okall = reduce_list([float(tot[:, 2].sum()), float(tot[:, 1].sum()), 1.0 if ok else 0.0],
                                       dist.ReduceOp.SUM)
    return {"workload": "C4 (BASELINE configs[3]): sin(1/x) on [1e-4,1] at EPSILON=1e-9, %d copies per pass as whole "
                        "integrals in contiguous blocks per rank, %d timed passes; and one integral per launch" % (m, reps),
            "value": leaves / elapsed, "unit": "accepted subintervals/s", "ms": elapsed * 1e3,
            "tasks_per_s": tasks / elapsed, "integrals_per_s": reps * m / elapsed,
            "single_integral_kernel_us": lone_us,
            "frac": None, "frac_note": "no algorithmic FLOP count is defined for glibc sin's range paths "
                                       "(SURVEY §8d defines 38 per task for cosh4 only)",
            "verified": okall == world,
            "checks": ["counts exact and areas to 1e-12 vs the golden sin(1/x) tree, every copy and the lone integral"]}


def c5_pass(ctx, rank, world, barrier, launch, reduce_list, dist, torch, all_reduce):
    """BASELINE configs[4]: EPSILON=1e-12, C5_COPIES copies of cosh4 on [0,5] in one launch, each
    integral sharded over the N GPUs; one untimed launch sizes the jobs, two are timed."""
    eps = 1e-12
    m = C5_COPIES
    launch(m, eps)                      # untimed
    ctx.synchronize()
    reps = 2
    totals = torch.zeros((reps * m, 4), dtype=torch.float64, device="cuda")
    ctx.kernel_timing(True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(reps):
        launch(m, eps)
        ctx.gather_results(0, m, totals.data_ptr() + i * m * 4 * totals.element_size())
    ctx.synchronize()
    all_reduce(totals, dist.ReduceOp.SUM)
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    kern_ms, launches = ctx.kernel_time()
    ctx.kernel_timing(False)
    tot = totals.cpu().numpy()
    tg, lg, ag = GOLDEN[eps]
    ok = bool((tot[:, 3] == 0).all() and (tot[:, 1] == tg).all() and (tot[:, 2] == lg).all()) and areas_ok(tot[:, 0], ag)
    elapsed, = reduce_list([t1 - t0], dist.ReduceOp.MAX)
    ksum, okall = reduce_list([kern_ms / 1e3, 1.0 if ok else 0.0], dist.ReduceOp.SUM)
    ok = okall == world
    tasks = float(tot[:, 1].sum())
    return {"workload": "C5 (BASELINE configs[4]): cosh4 on [0,5] at EPSILON=1e-12, %d copies per launch, each "
                        "sharded over the %d GPU(s), %d timed launches" % (m, world, reps),
            "value": float(tot[:, 2].sum()) / elapsed, "unit": "accepted subintervals/s", "ms": elapsed * 1e3,
            "frac": FLOP_PER_TASK * tasks / ksum / FP64_PEAK if ksum > 0 else None,
            "verified": ok, "checks": ["counts exact and areas to 1e-12 vs the golden tree, every copy"]}


if __name__ == "__main__":
    main()
