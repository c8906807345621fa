#!/bin/bash
# A/B sweep of the launch's job size (AQ_GSPLIT) and records per lane (AQ_ILP): one bench line per
# setting -> gpurun_out/sweep_<tag>.txt
set -euo pipefail
TAG=${1:-x}
OUT=gpurun_out/sweep_$TAG.txt
: > "$OUT"
for ilp in ${ILPS:-1 2}; do
  for gs in ${GSPLITS:-1 2 4 8}; do
    line=$(AQ_ILP=$ilp AQ_GSPLIT=$gs timeout -k 10 120 python bench.py --no-cpu-baseline --no-single --steps 512 --warmup 256)
    echo "ilp=$ilp gs=$gs $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_avg_us"], d["verified"])')" >> "$OUT"
  done
done
cat "$OUT"
