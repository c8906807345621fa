#!/bin/bash
# r06zf: small unsharded static launches deal ~W / k shares per integral (one job per wave) -- GPU suite,
# the small-launch sweep, sin(1/x) small launches
set -u
OUT=gpurun_out/r06zf; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc -ne 0 ] && exit $rc
sed 's#gpurun_out/r06zd#gpurun_out/r06zf#' tools/_r06zd.sh > /tmp/zd.sh && bash /tmp/zd.sh || exit 1
for n in libaquad_hb libaquad; do
  AQ_LIB=$PWD/ppls_amd/_build/$n.so timeout -k 10 200 python tools/try_sin_batch.py --k 1,2,4,8,11,12,16 --reps 5 > $OUT/sin_$n.json 2>&1 || { tail -3 $OUT/sin_$n.json; exit 1; }
  echo "$n $(tail -1 $OUT/sin_$n.json)"
done
