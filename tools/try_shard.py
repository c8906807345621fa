"""Strong-scaling rehearsal on ONE GPU (diagnostic tool): time rank 0's launch of K-integral batches
sharded N ways (what each of N GPUs runs in `bench.py --gpus N`), against 1/N of the unsharded
launch.  python tools/try_shard.py [--k 2048] [--reps 3]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ppls_amd import Context  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=2048, help="integrals per launch at 1 shard")
    ap.add_argument("--scale-k", action="store_true", help="N shards: N*k integrals per launch (bench.py's packing)")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--shards", default="1,2,4,8")
    args = ap.parse_args()
    ctx = Context(0)
    ctx.set_level_histograms(False)
    out = {"k": args.k, "scale_k": args.scale_k}
    base = base_tasks = None
    for n in [int(v) for v in args.shards.split(",")]:
        k = args.k * n if args.scale_k else args.k
        ctx.integrate_many_async(np.zeros(k), np.full(k, 5.0), 1e-10, shard=0, nshards=n)   # warmup
        ctx.synchronize()
        ctx.kernel_timing(True)
        for _ in range(args.reps):
            ctx.integrate_many_async(np.zeros(k), np.full(k, 5.0), 1e-10, shard=0, nshards=n)
        ctx.synchronize()
        ms, cnt = ctx.kernel_time()
        ctx.kernel_timing(False)
        us = ms * 1e3 / max(cnt, 1) * (args.k / k)   # per k integrals' worth of launches
        r = ctx.fetch(0)
        if base is None:
            base = us
        if base_tasks is None:
            base_tasks = r.tasks
        # rank 0 holds shard 0 of every integral here (the bench rotates shards over ranks), and shard 0
        # holds a little more or less than 1/N of each tree: the per-task rate is what the bench sees
        share = r.tasks * n / base_tasks
        out[f"shards{n}"] = {"kernel_us": us, "tasks_rank0": r.tasks, "rank0_task_share_x_n": share,
                             "efficiency_vs_1": base / (n * us), "efficiency_per_task": base * share / (n * us)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
