"""The bench's persistent launch and nothing else, for rocprofv3 kernel-trace / --pmc passes: one
untimed launch (sizes the jobs), then --reps launches of --k copies of cosh4 on [0,5] at --eps through
the batch front end (one launch, one device gather and one copy each -- a handful of dispatches per
launch, where per-slot fetches would add tens of thousands of copy kernels to the counter CSVs).
Every integral's counts are checked against the golden tree. Prints one JSON line. Diagnostic tool.

  python tools/pmc_bench_launch.py [--k 32768] [--reps 2] [--eps 1e-10]
"""
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
    ap.add_argument("--k", type=int, default=32768)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--eps", type=float, default=1e-10)
    args = ap.parse_args()
    trees = json.load(open(os.path.join(ROOT, "tests", "golden", "trees.json")))
    g = trees[{1e-10: "cosh4_eps1e-10", 1e-12: "cosh4_eps1e-12", 1e-8: "cosh4_eps1e-8", 1e-3: "cosh4_eps1e-3"}[args.eps]]
    ctx = Context(0)
    ctx.set_level_histograms(False)
    a, b = np.zeros(args.k), np.full(args.k, 5.0)
    ctx.integrate_batch(a, b, args.eps)
    ctx.synchronize()
    ok = True
    ctx.kernel_timing(True)
    for _ in range(args.reps):
        _, tasks, acc = ctx.integrate_batch(a, b, args.eps)
        ok = ok and bool((tasks == g["tasks"]).all() and (acc == g["leaves"]).all())
    ms, n = ctx.kernel_time()
    ctx.kernel_timing(False)
    print(json.dumps({"k": args.k, "eps": args.eps, "reps": args.reps, "counts_ok": ok, "kernel_us": ms * 1e3 / max(n, 1),
                      "tasks_per_launch": args.k * g["tasks"], "accepted_per_launch": args.k * g["leaves"]}))
    ctx.close()


if __name__ == "__main__":
    main()
