#!/bin/bash
# r06zo: the batch's scatter of chunks c >= 1 in order on the launch stream (behind the previous gather,
# after a wait on the estimate) against it on the pre-pass stream (libaquad_sc0) -- GPU suite, C3 A/B
set -u
OUT=gpurun_out/r06zo; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc -ne 0 ] && exit $rc
ROUNDS=4 SINGLE=0 LIBS="libaquad_sc0 libaquad" bash tools/ab_c3.sh r06zo > "$OUT/ab_c3.txt" 2>&1 || { tail -5 "$OUT/ab_c3.txt"; exit 1; }
cat "$OUT/ab_c3.txt"
