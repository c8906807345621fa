#!/bin/bash
# sin(1/x) A/B of library variants (ppls_amd/_build/libaquad_*.so): tools/try_sin_batch.py per variant.
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/absin_$TAG
mkdir -p "$OUT"
for r in $(seq 1 ${ROUNDS:-2}); do
  for so in ppls_amd/_build/libaquad_*.so; do
    n=$(basename "$so" .so)
    AQ_LIB=$PWD/$so timeout -k 10 120 python tools/try_sin_batch.py > "$OUT/$n.$r.json" 2> "$OUT/$n.$r.err" || { echo "$n failed"; tail -5 "$OUT/$n.$r.err"; exit 1; }
    echo "$r $n $(cat "$OUT/$n.$r.json")"
  done
done
