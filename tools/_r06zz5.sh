#!/bin/bash
# r06zz5: HEAD against the r06zn-era library on one box (bench launch + lone, 3 alternating passes)
set -u
OUT=gpurun_out/r06zz5; mkdir -p $OUT
ROUNDS=3 K=32768 REPS=2 SINGLE=20 C3=0 AB_GLOB="libaquad*.so" bash tools/ab.sh r06zz5 > $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
python3 - <<'PY'
import json,glob,collections
res=collections.defaultdict(list)
for f in sorted(glob.glob('gpurun_out/ab_r06zz5/libaquad*.[0-9].json')):
    n=f.split('/')[-1].rsplit('.',2)[0]
    try: res[n].append(json.load(open(f)))
    except Exception: pass
for n,v in res.items():
    print(n, 'bench_launch_us', [round(x['kernel_us']) for x in v if 'kernel_us' in x], 'lone_us', [round(x['single_us'],2) for x in v if 'single_us' in x])
PY
