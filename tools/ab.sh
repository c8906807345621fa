#!/bin/bash
# Alternating A/B of library variants on one GPU box: ROUNDS passes over every
# ppls_amd/_build/${AB_GLOB:-libaquad_*.so} (built here with `python ppls_amd/build.py --variant NAME -D...`),
# one process per run, so order effects and box drift show up as pass-to-pass spread.
#   tools/ab.sh <tag>        (env: ROUNDS=3 K=8192 EPS=1e-10 REPS=3 SINGLE=20 C3=65536)
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/ab_$TAG
mkdir -p "$OUT"
for r in $(seq 1 ${ROUNDS:-3}); do
  for so in ppls_amd/_build/${AB_GLOB:-libaquad_*.so}; do
    n=$(basename "$so" .so)
    AQ_LIB=$PWD/$so timeout -k 10 180 python tools/try_kernel.py --k ${K:-8192} --eps ${EPS:-1e-10} --reps ${REPS:-3} \
        --single ${SINGLE:-20} --c3 ${C3:-65536} > "$OUT/$n.$r.json" 2> "$OUT/$n.$r.err" || { echo "$n failed"; tail -5 "$OUT/$n.$r.err"; exit 1; }
    echo "$r $n $(cat "$OUT/$n.$r.json")"
  done
done
