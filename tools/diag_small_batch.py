import sys, time, json
sys.path.insert(0, '/root/repo')
import numpy as np
from ppls_amd import Context
from tools.bench_batch import splitmix64_bounds
ctx = Context(0); ctx.set_level_histograms(False)
a, b = splitmix64_bounds(16384)
out = {}
for eps in (1e-3, 1e-10):
    for k in (2048, 16384):
        ctx.integrate_many_async(a[:k], b[:k], eps); ctx.synchronize()
        ctx.kernel_timing(True)
        t0 = time.perf_counter()
        for _ in range(3):
            ctx.integrate_many_async(a[:k], b[:k], eps)
        ctx.synchronize()
        t1 = time.perf_counter()
        ms, n = ctx.kernel_time(); ctx.kernel_timing(False)
        out[f"{eps:g}_k{k}"] = {"kernel_ms": ms / n, "wall_ms": (t1 - t0) * 1e3 / 3}
    t0 = time.perf_counter(); ctx.integrate_batch(a, b, eps); t1 = time.perf_counter()
    out[f"{eps:g}_batch16384_wall_ms"] = (t1 - t0) * 1e3
print(json.dumps(out, indent=1))
