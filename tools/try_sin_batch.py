"""Kernel time of sin(1/x) batches (BASELINE config 4's integrand) for A/B of library variants
(diagnostic tool; loads the library named by AQ_LIB). Counts checked against the golden tree.

  python tools/try_sin_batch.py [--k 1,64,4096] [--reps 5]     -> one JSON line: us per launch per K
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ppls_amd import SIN_RECIP, Context  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", default="1,64,4096")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "trees.json")))["sin_recip_eps1e-9"]
    out = {"lib": os.environ.get("AQ_LIB", "default")}
    with Context(0) as ctx:
        ctx.set_level_histograms(False)
        for k in (int(v) for v in args.k.split(",")):
            a, b = np.full(k, 1e-4), np.full(k, 1.0)
            ctx.integrate_many_async(a, b, 1e-9, integrand=SIN_RECIP)   # warmup (and the job-size hint)
            ctx.synchronize()
            ctx.kernel_timing(True)
            for _ in range(args.reps):
                ctx.integrate_many_async(a, b, 1e-9, integrand=SIN_RECIP)
            ctx.synchronize()
            ms, n = ctx.kernel_time()
            ctx.kernel_timing(False)
            ok = all((ctx.fetch(i).tasks, ctx.fetch(i).accepted) == (g["tasks"], g["leaves"]) for i in (0, k - 1))
            out["k%d_us" % k] = round(ms * 1e3 / max(n, 1), 2)
            out["k%d_ok" % k] = ok
    print(json.dumps(out))


if __name__ == "__main__":
    main()
