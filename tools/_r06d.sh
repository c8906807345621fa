#!/bin/bash
# r06d: per-CU area in per-workgroup words (PCU_AREA) + heap-order seeding of whole-integral jobs: GPU suite,
# then C3 (eps=1e-3) and lone A/B against the r06a code (x0base) and against no heap seeding (x5noheap),
# and the synchronous call's wall latency for base and new.
set -u
TAG=r06d
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc -ne 0 ] && exit $rc
ROUNDS=3 LIBS="libaquad_x0base libaquad libaquad_x5noheap" bash tools/ab_c3.sh $TAG > "$OUT/ab_c3.txt" 2>&1 || { tail -5 "$OUT/ab_c3.txt"; exit 1; }
cat "$OUT/ab_c3.txt"
for n in libaquad_x0base libaquad; do
  AQ_LIB=$PWD/ppls_amd/_build/$n.so timeout -k 10 120 python tools/try_wall.py > "$OUT/wall_$n.json" 2>&1 || exit 1
  echo "$n wall $(cat $OUT/wall_$n.json)"
done
