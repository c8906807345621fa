"""Wall and kernel time of aq_integrate_batch across batch sizes and tolerances (C3 splitmix64 bounds),
beside the same integrals as one aq_integrate_many_async launch where they fit (diagnostic tool).

  python tools/batch_sizes.py [--n 64,512,4096,32768,262144] [--eps 1e-3,1e-8] [--reps 3] [--sin]
(--sin: sin(1/x), config 4's integrand, on the C3 bounds mapped into [1e-4, 1])
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ppls_amd import SIN_RECIP, Context  # noqa: E402
from tools.bench_batch import splitmix64_bounds  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="64,512,4096,32768,262144")
    ap.add_argument("--eps", default="1e-3,1e-8")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--sin", action="store_true")
    args = ap.parse_args()
    f = SIN_RECIP if args.sin else 0
    ctx = Context(0)
    ctx.set_level_histograms(False)
    out = []
    for eps in (float(e) for e in args.eps.split(",")):
        for n in (int(v) for v in args.n.split(",")):
            a, b = splitmix64_bounds(n)
            if args.sin:
                a, b = 1e-4 + a * (1.0 - 1e-4) / 5.0, 1e-4 + b * (1.0 - 1e-4) / 5.0 + 1e-6
            ctx.integrate_batch(a, b, eps, integrand=f)   # warm (hint, pool, buffers)
            walls, kms = [], []
            for _ in range(args.reps):
                ctx.synchronize()
                ctx.kernel_timing(True)
                t0 = time.perf_counter()
                _, tasks, acc = ctx.integrate_batch(a, b, eps, integrand=f)
                walls.append((time.perf_counter() - t0) * 1e3)
                kms.append(ctx.kernel_time()[0])
                ctx.kernel_timing(False)
            rec = {"integrand": "sin_recip" if args.sin else "cosh4", "eps": eps, "n": n, "batch_wall_ms": round(min(walls), 3), "batch_kernel_ms": round(min(kms), 3),
                   "tasks": int(tasks.sum()), "t_eq_2l_1": bool((tasks == 2 * acc - 1).all())}
            if n <= ctx.max_integrals_per_launch:
                ctx.integrate_many_async(a, b, eps, first_slot=0, integrand=f)
                ctx.synchronize()
                ctx.kernel_timing(True)
                for _ in range(args.reps):
                    ctx.integrate_many_async(a, b, eps, first_slot=0, integrand=f)
                ms, k = ctx.kernel_time()
                ctx.kernel_timing(False)
                rec["many_kernel_ms"] = round(ms / max(k, 1), 3)
            out.append(rec)
            print(json.dumps(rec), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
