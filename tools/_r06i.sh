#!/bin/bash
# r06i: heap seeding as the batch front end's own k_stream instance -- GPU suite, then the bench launch
# (32768 x cosh4 eps=1e-10) and lone, and C3 eps=1e-3 through aq_integrate_batch, HEAD against the r06b code
set -u
OUT=gpurun_out/r06i; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc -ne 0 ] && exit $rc
ROUNDS=3 K=32768 REPS=2 SINGLE=20 C3=0 AB_GLOB="libaquad*.so" bash tools/ab.sh r06i > $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
ROUNDS=3 SINGLE=0 LIBS="libaquad_r06b libaquad" bash tools/ab_c3.sh r06i > $OUT/ab_c3.txt 2>&1 || { tail -5 $OUT/ab_c3.txt; exit 1; }
python3 - <<'PY'
import json,glob,collections
res=collections.defaultdict(list)
for f in sorted(glob.glob('gpurun_out/ab_r06i/*.[0-9].json')):
    n=f.split('/')[-1].rsplit('.',2)[0]; d=json.load(open(f)); res[n].append(d)
for n,v in res.items():
    print(n, 'bench_us', [round(x['kernel_us']) for x in v], 'single', [round(x['single_us'],2) for x in v], all(x['bench_ok'] and x['single_ok'] and x['batch256_ok'] for x in v))
PY
cat $OUT/ab_c3.txt
