#!/bin/bash
# single-integral latency (K=1 launches) across library variants (ppls_amd/_build/libaquad_*.so)
mkdir -p gpurun_out/abs
for so in ppls_amd/_build/libaquad*.so; do
  n=$(basename $so .so)
  AQ_LIB=$PWD/$so timeout -k 10 120 python tools/try_engine.py --engine stream --reps ${REPS:-20} --k 1 --eps ${EPS:-1e-10} > gpurun_out/abs/$n.json 2>&1 || { echo "$n failed"; continue; }
  echo "$n $(python3 -c "import json;d=json.load(open('gpurun_out/abs/$n.json'));print(d['bench_ok'], round(d['kernel_us'],1))")"
done
