"""a batch of 1 000 000 independent cos h^4 integrals with splitmix64 bounds
on one MI355X, through the batch front end (aq_integrate_batch: 65536-integral persistent launches,
device gathers, one host sync). Prints accepted subintervals/s and the KAT of §8d (mean leaves of
the first 10 000 draws: 711.5 at eps=1e-3, 153 330.8 at eps=1e-10).

  python tools/bench_batch.py [--n 1000000] [--eps 1e-3,1e-10] [--reps 1]
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

KAT = {1e-3: 711.5, 1e-10: 153330.8}
GOLDEN = 0x9E3779B97F4A7C15


def splitmix64_bounds(n):
    """state += golden; standard mix; u = (z >> 11) * 2^-53; a = 5u1, b = 5u2, swap."""
    with np.errstate(over="ignore"):
        k = np.arange(1, 2 * n + 1, dtype=np.uint64)
        z = np.uint64(GOLDEN) + k * np.uint64(GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
    a, b = 5.0 * u[0::2], 5.0 * u[1::2]
    return np.minimum(a, b), np.maximum(a, b)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--eps", default="1e-3,1e-10")
    ap.add_argument("--reps", type=int, default=1)
    args = ap.parse_args()
    ctx = Context(0)
    ctx.set_level_histograms(False)
    a, b = splitmix64_bounds(args.n)
    out = {"n": args.n}
    for eps in [float(e) for e in args.eps.split(",")]:
        ctx.integrate_batch(a[:65536], b[:65536], eps)          # warmup
        best = None
        for _ in range(args.reps):
            t0 = time.perf_counter()
            area, tasks, acc = ctx.integrate_batch(a, b, eps)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        leaves = int(acc.sum())
        kat = round(float(acc[:10000].mean()), 1)
        out[f"eps{eps:g}"] = {
            "seconds": best, "leaves": leaves, "tasks": int(tasks.sum()),
            "accepted_per_s": leaves / best, "integrals_per_s": args.n / best,
            "kat_mean_leaves_first10000": kat, "kat_expected": KAT.get(eps),
            "kat_ok": (KAT.get(eps) is None) or kat == KAT[eps],
            "tasks_eq_2L_minus_1": bool((tasks == 2 * acc - 1).all()),
        }
        print(json.dumps({f"eps{eps:g}": out[f"eps{eps:g}"]}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
