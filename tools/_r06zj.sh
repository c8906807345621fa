#!/bin/bash
# r06zj: sin(1/x) with a correctly rounded reciprocal sequence (recip_rn) -- GPU suite (incl. the
# bit-exact device sin(1/x) check), then sin batches and the lone sin against HEAD (libaquad_hb)
set -u
OUT=gpurun_out/r06zj; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for n in libaquad_hb libaquad; do
    AQ_LIB=$PWD/ppls_amd/_build/$n.so timeout -k 10 200 python tools/try_sin_batch.py --k 1,64,4096 --reps 8 > $OUT/sin_$n.$r.json 2>&1 || { tail -3 $OUT/sin_$n.$r.json; exit 1; }
    echo "$r $n $(tail -1 $OUT/sin_$n.$r.json)"
  done
done
