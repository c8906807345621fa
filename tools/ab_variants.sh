#!/bin/bash
# A/B the persistent kernel across library variants (ppls_amd/_build/libaquad_*.so), one process each.
mkdir -p gpurun_out/ab
for so in ppls_amd/_build/libaquad*.so; do
  n=$(basename $so .so)
  AQ_LIB=$PWD/$so timeout -k 10 120 python tools/try_engine.py --engine ${ENGINE:-stream} --reps ${REPS:-2} --k ${K:-2048} > gpurun_out/ab/$n.json 2>&1 || { echo "$n failed"; exit 1; }
  echo "$n $(python3 -c "import json;d=json.load(open('gpurun_out/ab/$n.json'));print(d['bench_ok'], round(d['kernel_us'],1), '%.3e'%d['accepted_per_s_kernel'])")"
done
