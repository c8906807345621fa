"""Kernel time of one maximum-size batch launch (262144 splitmix64 integrals, the C3 bounds) at a
1-task tree per integral (eps=1e30: the per-integral fixed cost -- seeding, flush, job claims), at
eps=1e-1 and at C3's eps=1e-3 (~1 420 tasks per integral). HIP events, mean of 3 launches.
    python tools/try_tiny.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ppls_amd import Context  # noqa: E402
from tools.bench_batch import splitmix64_bounds  # noqa: E402


def main():
    ctx = Context(0)
    ctx.set_level_histograms(False)
    k = 262144
    a, b = splitmix64_bounds(k)
    out = {"lib": os.environ.get("AQ_LIB", "default"), "integrals": k}
    for eps in (1e30, 1e-1, 1e-3):
        ctx.integrate_many_async(a, b, eps)
        ctx.synchronize()
        ctx.kernel_timing(True)
        for _ in range(3):
            ctx.integrate_many_async(a, b, eps)
        ctx.synchronize()
        ms, n = ctx.kernel_time()
        ctx.kernel_timing(False)
        out["eps%g" % eps] = {"kernel_ms": round(ms / n, 4), "ns_per_integral": round(ms / n * 1e6 / k, 2)}
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
