#!/bin/bash
# r06j: loop alignment of the device code (-falign-loops=32/64/128 against the default) on the bench launch
set -u
OUT=gpurun_out/r06j; mkdir -p $OUT
ROUNDS=3 K=32768 REPS=2 SINGLE=20 C3=0 AB_GLOB="libaquad*.so" bash tools/ab.sh r06j > $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
python3 - <<'PY'
import json,glob,collections
res=collections.defaultdict(list)
for f in sorted(glob.glob('gpurun_out/ab_r06j/libaquad*.[0-9].json')):
    n=f.split('/')[-1].rsplit('.',2)[0]; res[n].append(json.load(open(f)))
for n,v in res.items():
    print(n, 'bench_launch_us', [round(x['kernel_us']) for x in v], 'lone_us', [round(x['single_us'],2) for x in v], 'ok', all(x['bench_ok'] and x['single_ok'] for x in v))
PY
