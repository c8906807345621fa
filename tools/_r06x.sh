#!/bin/bash
# r06x: launches of few integrals take up to one job per wave (MIN_JOB_TASKS) -- GPU suite, then
# sin(1/x) and cosh4 batches of 16 .. 4096 integrals and the bench launch against HEAD (libaquad_hb)
set -u
OUT=gpurun_out/r06x; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for n in libaquad_hb libaquad; do
    AQ_LIB=$PWD/ppls_amd/_build/$n.so timeout -k 10 200 python tools/try_sin_batch.py --k 16,64,256,1024,4096 --reps 5 > $OUT/sin_$n.$r.json 2>&1 || { tail -3 $OUT/sin_$n.$r.json; exit 1; }
    echo "$r $n sin $(tail -1 $OUT/sin_$n.$r.json)"
  done
done
ROUNDS=2 K=32768 REPS=2 SINGLE=20 C3=0 AB_GLOB="libaquad*.so" bash tools/ab.sh r06x > $OUT/ab.txt 2>&1 || { tail -5 $OUT/ab.txt; exit 1; }
python3 - <<'PY'
import json,glob,collections
res=collections.defaultdict(list)
for f in sorted(glob.glob('gpurun_out/ab_r06x/libaquad*.[0-9].json')):
    n=f.split('/')[-1].rsplit('.',2)[0]; res[n].append(json.load(open(f)))
for n,v in res.items():
    print(n, 'bench_launch_us', [round(x['kernel_us']) for x in v], 'lone_us', [round(x['single_us'],2) for x in v], 'ok', all(x['bench_ok'] and x['single_ok'] for x in v))
PY
