"""Kernel A/B probe on the GPU (diagnostic tool; loads the library named by AQ_LIB, default the
in-tree build). Checks parity on small cases, then times the three shapes that matter:
  * the bench launch: K integrals of cosh4 [0,5] per launch at --eps (default 8192 at 1e-10),
  * a lone integral (aq_integrate-shaped launches, K=1),
  * a C3-like batch of random bounds at eps=1e-3 (--c3 N integrals, launch-bound).
Prints one JSON object.  python tools/try_kernel.py [--k 8192] [--reps 3] [--single 20] [--c3 65536]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ppls_amd import Context, Problem  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--eps", type=float, default=1e-10)
    ap.add_argument("--single", type=int, default=20)
    ap.add_argument("--c3", type=int, default=65536)
    args = ap.parse_args()
    trees = json.load(open(os.path.join(ROOT, "tests", "golden", "trees.json")))
    batch = json.load(open(os.path.join(ROOT, "tests", "golden", "batch.json")))
    from tools.bench_batch import splitmix64_bounds   # the C3 generator (no oracle in tools/)
    ctx = Context(0)
    ctx.set_level_histograms(False)
    out = {"lib": os.environ.get("AQ_LIB", "default")}
    g3 = trees["cosh4_eps1e-3"]
    ctx.integrate_many_async(np.zeros(32), np.full(32, 5.0), 1e-3)
    out["eps1e-3_x32_ok"] = all((r.tasks, r.accepted) == (g3["tasks"], g3["leaves"]) for r in (ctx.fetch(i) for i in range(32)))
    a, b = splitmix64_bounds(max(256, args.c3))
    ctx.integrate_many_async(a[:256], b[:256], 1e-3)
    out["batch256_ok"] = [ctx.fetch(i).accepted for i in range(256)] == batch["leaves_eps1e-3_first256"]
    tag = {1e-10: "cosh4_eps1e-10", 1e-12: "cosh4_eps1e-12", 1e-8: "cosh4_eps1e-8", 1e-6: "cosh4_eps1e-6",
           1e-3: "cosh4_eps1e-3"}[args.eps]
    g = trees[tag]
    k = args.k
    ctx.integrate_many_async(np.zeros(k), np.full(k, 5.0), args.eps)
    ctx.synchronize()
    ctx.kernel_timing(True)
    for _ in range(args.reps):
        ctx.integrate_many_async(np.zeros(k), np.full(k, 5.0), args.eps)
    ms, n = ctx.kernel_time()
    ctx.kernel_timing(False)
    rs = [ctx.fetch(i) for i in range(k)]
    out["bench_ok"] = all((r.tasks, r.accepted) == (g["tasks"], g["leaves"]) for r in rs)
    out["kernel_us"] = ms * 1e3 / max(n, 1)
    out["accepted_per_s_kernel"] = g["leaves"] * k / (ms * 1e-3 / max(n, 1))
    if args.single:
        p = Problem(eps=args.eps)
        ctx.integrate_async(p, 0)
        ctx.synchronize()
        ctx.kernel_timing(True)
        for _ in range(args.single):
            ctx.integrate_async(p, 0)
        ms1, n1 = ctx.kernel_time()
        ctx.kernel_timing(False)
        r = ctx.fetch(0)
        out["single_ok"] = (r.tasks, r.accepted) == (g["tasks"], g["leaves"])
        out["single_us"] = ms1 * 1e3 / max(n1, 1)
    if args.c3:
        m = args.c3
        ctx.integrate_many_async(a[:m], b[:m], 1e-3)
        ctx.synchronize()
        t0 = time.perf_counter()
        ctx.kernel_timing(True)
        ctx.integrate_many_async(a[:m], b[:m], 1e-3)
        ms3, _ = ctx.kernel_time()
        ctx.kernel_timing(False)
        out["c3_eps1e-3_kernel_us"] = ms3 * 1e3
        out["c3_wall_ms"] = (time.perf_counter() - t0) * 1e3
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
