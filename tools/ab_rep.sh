#!/bin/bash
# Alternating A/B of the library variants (ppls_amd/_build/libaquad*.so): ROUNDS passes over all
# variants in turn (order effects and box drift show up as pass-to-pass spread), K integrals per launch.
mkdir -p gpurun_out/abr
for r in $(seq 1 ${ROUNDS:-3}); do
  for so in ppls_amd/_build/libaquad*.so; do
    n=$(basename $so .so)
    AQ_LIB=$PWD/$so timeout -k 10 120 python tools/try_engine.py --engine stream --reps ${REPS:-2} --k ${K:-8192} > gpurun_out/abr/$n.$r.json 2>&1 || { echo "$n failed"; exit 1; }
    echo "$r $n $(python3 -c "import json;d=json.load(open('gpurun_out/abr/$n.$r.json'));print(d['bench_ok'], round(d['kernel_us'],1), '%.3e'%d['accepted_per_s_kernel'])")"
  done
done
