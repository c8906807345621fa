#!/bin/bash
# r06h: the bench launch (32768 x cosh4 eps=1e-10), lone and C3 probes across: HEAD (libaquad), HEAD without
# heap seeding (noheap), and the r06b code (before the per-CU area words and heap seeding)
set -u
ROUNDS=3 K=32768 REPS=2 SINGLE=20 C3=262144 AB_GLOB="libaquad*.so" bash tools/ab.sh r06h > gpurun_out/ab_r06h.txt 2>&1 || { tail -5 gpurun_out/ab_r06h.txt; exit 1; }
python3 - <<'PY'
import json,glob,collections
res=collections.defaultdict(list)
for f in sorted(glob.glob('gpurun_out/ab_r06h/*.json')):
    n=f.split('/')[-1].rsplit('.',2)[0]; d=json.load(open(f)); res[n].append(d)
for n,v in res.items():
    print(n, 'bench_us', [round(x['kernel_us']) for x in v], 'single', [round(x['single_us'],2) for x in v], 'c3', [round(x['c3_eps1e-3_kernel_us']) for x in v], all(x['bench_ok'] and x['single_ok'] and x['batch256_ok'] for x in v))
PY
