#!/bin/bash
# r06za: GPU suite, then the cosh4 few-integral sweep (tools/_r06z.sh) and sin(1/x) batches against
# the code before the fill rule (libaquad_hb)
set -u
OUT=gpurun_out/r06za; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc -ne 0 ] && exit $rc
bash tools/_r06z.sh || exit 1
for n in libaquad_hb libaquad; do
  AQ_LIB=$PWD/ppls_amd/_build/$n.so timeout -k 10 200 python tools/try_sin_batch.py --k 16,64,256,1024,4096 --reps 5 > $OUT/sin_$n.json 2>&1 || { tail -3 $OUT/sin_$n.json; exit 1; }
  echo "$n sin $(tail -1 $OUT/sin_$n.json)"
done
