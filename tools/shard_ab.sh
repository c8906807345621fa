#!/bin/bash
# A/B of library variants on rank 0's sharded launch (tools/try_shard.py --scale-k: N x K integrals
# sharded N ways, against 1/N of the unsharded launch), ROUNDS passes over every
# ppls_amd/_build/${AB_GLOB:-libaquad_*.so}.   tools/shard_ab.sh <tag>   (env: ROUNDS=2 K=16384)
set -o pipefail
OUT=gpurun_out/shard_ab_${1:?tag}
mkdir -p "$OUT"
for r in $(seq 1 ${ROUNDS:-2}); do
  for so in ppls_amd/_build/${AB_GLOB:-libaquad_*.so}; do
    v=$(basename "$so" .so)
    AQ_LIB=$PWD/$so timeout -k 10 120 python tools/try_shard.py --scale-k --k ${K:-16384} --reps 3 > "$OUT/$v.$r.json" 2> "$OUT/$v.$r.err" \
      || { echo "$v failed"; tail -5 "$OUT/$v.$r.err"; exit 1; }
    echo "$r $v $(python -c "import json; d=json.load(open('$OUT/$v.$r.json')); print({k: round(v['kernel_us']) for k, v in d.items() if k.startswith('shards')})")"
  done
done
