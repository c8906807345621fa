"""Kernel time of one C3-shaped launch (splitmix64 bounds, eps=1e-3) against its integral count: the
fit t = fixed + per-integral x k separates a launch's fixed cost (ramp, tail) from its work.
Diagnostic tool.  python tools/c3_launch_sizes.py [--reps 3]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ppls_amd import Context  # noqa: E402
from tools.bench_batch import splitmix64_bounds  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--eps", type=float, default=1e-3)
    args = ap.parse_args()
    ctx = Context(0)
    ctx.set_level_histograms(False)
    a, b = splitmix64_bounds(262144)
    out = {"lib": os.environ.get("AQ_LIB", "default"), "eps": args.eps, "us": {}}
    for k in (4096, 8192, 16384, 32768, 65536, 131072, 262144):
        ctx.integrate_many_async(a[:k], b[:k], args.eps)
        ctx.synchronize()
        ctx.kernel_timing(True)
        for _ in range(args.reps):
            ctx.integrate_many_async(a[:k], b[:k], args.eps)
        ms, n = ctx.kernel_time()
        ctx.kernel_timing(False)
        out["us"][k] = ms * 1e3 / n
    ks = sorted(out["us"])
    import numpy as np
    A = np.vstack([np.ones(len(ks)), np.array(ks, float)]).T
    fixed, per = np.linalg.lstsq(A, np.array([out["us"][k] for k in ks]), rcond=None)[0]
    out["fit"] = {"fixed_us": fixed, "per_integral_ns": per * 1e3}
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
