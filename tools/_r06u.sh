#!/bin/bash
# r06u: 256 size classes (8 per octave) for the batch's size order -- GPU suite, then C3 at eps=1e-3 and
# 1e-10 against the 64-class code (libaquad_k64), alternating
set -u
OUT=gpurun_out/r06u; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc -ne 0 ] && exit $rc
ROUNDS=3 SINGLE=0 LIBS="libaquad_k64 libaquad" bash tools/ab_c3.sh r06u > "$OUT/ab_c3.txt" 2>&1 || { tail -5 "$OUT/ab_c3.txt"; exit 1; }
cat "$OUT/ab_c3.txt"
ROUNDS=2 SINGLE=0 EPS=1e-10 LIBS="libaquad_k64 libaquad" bash tools/ab_c3.sh r06u10 > "$OUT/ab_c3_1e10.txt" 2>&1 || { tail -5 "$OUT/ab_c3_1e10.txt"; exit 1; }
cat "$OUT/ab_c3_1e10.txt"
