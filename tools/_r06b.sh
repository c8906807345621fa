#!/bin/bash
# r06b: the ADVICE-r5 changes on the GPU (full suite, smoke, bench with the warmed column sum), then a
# lone-integral A/B of timing variants of the per-CU exit (area fold / cu counter atomics skipped).
set -u
TAG=r06b
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
bash tools/r05_final.sh $TAG || exit $?
ROUNDS=3 bash tools/ab_single.sh $TAG > "$OUT/ab_single.txt" 2>&1 || { tail -5 "$OUT/ab_single.txt"; exit 1; }
cat "$OUT/ab_single.txt"
