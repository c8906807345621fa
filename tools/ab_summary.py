"""Summarise tools/ab.sh output: per variant the median bench-launch kernel time, accepted/s, lone
integral and C3 eps=1e-3 kernel times, and whether every parity check passed.
  python tools/ab_summary.py gpurun_out/ab_<tag>"""
import glob
import json
import os
import statistics
import sys

rows = {}
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    name = os.path.basename(f).rsplit(".", 2)[0]
    try:
        d = json.load(open(f))
    except Exception:
        continue
    rows.setdefault(name, []).append(d)
base = None
for name, ds in sorted(rows.items()):
    k = statistics.median(d["kernel_us"] for d in ds)
    base = base or k
    ok = all(d.get("bench_ok") and d.get("eps1e-3_x32_ok") and d.get("batch256_ok") and d.get("single_ok", True) for d in ds)
    single = statistics.median(d.get("single_us", 0) for d in ds)
    c3 = statistics.median(d.get("c3_eps1e-3_kernel_us", 0) for d in ds)
    print(f"{name:28s} kernel {k:9.1f} us ({(k / base - 1) * 100:+5.1f}%)  {statistics.median(d['accepted_per_s_kernel'] for d in ds):.4e}/s"
          f"  single {single:6.1f} us  c3 {c3:7.1f} us  n={len(ds)} ok={ok}")
