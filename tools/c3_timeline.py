"""Where the C3 (BASELINE configs[2]) wall time goes: 1 M splitmix64-bounded integrals at --eps through
aq_integrate_batch, timed as the bench's secondary pass times it (wall) beside the HIP-event time of
its persistent launches. Run under `rocprofv3 --kernel-trace --memory-copy-trace` for the device
timeline (tools/c3_timeline_summary.py folds the CSVs). Diagnostic tool.

  python tools/c3_timeline.py [--eps 1e-3] [--n 1000000] [--reps 3] [--reuse-out]
  (AQ_BATCH_TRACE=1: the library prints each call's host phase times on stderr)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ppls_amd import Context  # noqa: E402
from tools.bench_batch import splitmix64_bounds  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--eps", type=float, default=1e-3)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--reuse-out", action="store_true", help="write every call into the same output arrays")
    args = ap.parse_args()
    ctx = Context(0)
    ctx.set_level_histograms(False)
    a, b = splitmix64_bounds(args.n)
    ctx.integrate_batch(a[:65536], b[:65536], args.eps)   # sizes the jobs (launch-to-launch hint)
    out = {"eps": args.eps, "n": args.n, "reuse_out": args.reuse_out, "reps": []}
    bufs = (np.zeros(args.n), np.zeros(args.n, np.uint64), np.zeros(args.n, np.uint64)) if args.reuse_out else None
    for _ in range(args.reps):
        ctx.synchronize()
        ctx.kernel_timing(True)
        t0 = time.perf_counter()
        area, tasks, acc = ctx.integrate_batch(a, b, args.eps, out=bufs)
        t1 = time.perf_counter()
        ms, n = ctx.kernel_time()
        ctx.kernel_timing(False)
        out["reps"].append({"wall_ms": (t1 - t0) * 1e3, "kernel_ms": ms, "launches": n,
                            "tasks": int(tasks.sum()), "accepted": int(acc.sum()),
                            "t_eq_2l_1": bool((tasks == 2 * acc - 1).all())})
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
