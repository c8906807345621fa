#!/bin/bash
# r06zs/zt: claim runs capped by the hint's tasks per integral, first jobs dealt transposed (HEAPS) -- GPU suite, batch sizes at
# eps=1e-8 / 1e-3 against HEAD (libaquad_hb), the unsorted batch beside, and C3 eps=1e-3
set -u
OUT=gpurun_out/r06zs; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for n in libaquad_hb libaquad; do
    AQ_LIB=$PWD/ppls_amd/_build/$n.so timeout -k 10 300 python tools/batch_sizes.py --n 4096,32768,262144 --eps 1e-8,1e-3 > $OUT/$n.$r.jsonl 2> $OUT/$n.$r.err || { tail -3 $OUT/$n.$r.err; exit 1; }
    echo "$r $n"; cat $OUT/$n.$r.jsonl
  done
done
AQ_BATCH_SORT=0 timeout -k 10 300 python tools/batch_sizes.py --n 4096,262144 --eps 1e-8 > $OUT/nosort.jsonl 2> $OUT/nosort.err || { tail -3 $OUT/nosort.err; exit 1; }
echo nosort; cat $OUT/nosort.jsonl
ROUNDS=2 SINGLE=0 LIBS="libaquad_hb libaquad" bash tools/ab_c3.sh r06zs > "$OUT/ab_c3.txt" 2>&1 || { tail -5 "$OUT/ab_c3.txt"; exit 1; }
cat "$OUT/ab_c3.txt"
