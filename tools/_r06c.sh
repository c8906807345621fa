#!/bin/bash
# r06c: per-CU area fold moved to the waiting leaders -- GPU suite + smoke, then lone A/B against the
# r06a code (x0base).
set -u
TAG=r06c
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc -ne 0 ] && exit $rc
ROUNDS=3 bash tools/ab_single.sh $TAG > "$OUT/ab_single.txt" 2>&1 || { tail -5 "$OUT/ab_single.txt"; exit 1; }
cat "$OUT/ab_single.txt"
