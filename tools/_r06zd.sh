#!/bin/bash
# r06zd: kernel time across the launch-size regimes around the static / adaptive boundary
# (k = 2, 8, 11 per-CU static; 12, 15 static; 16, 24, 32 adaptive with the fill rule), cosh4 [0,5]
set -u
OUT=gpurun_out/r06zd; mkdir -p $OUT
for eps in 1e-10 1e-8; do
  for k in 1 2 8 11 12 15 16 24 32; do
    timeout -k 10 120 python tools/try_kernel.py --k $k --eps $eps --reps 3 --single 0 --c3 0 > $OUT/$eps.$k.json 2> $OUT/$eps.$k.err || { tail -3 $OUT/$eps.$k.err; exit 1; }
    echo "eps=$eps k=$k $(python3 -c "import json;d=json.load(open('$OUT/$eps.$k.json'));print(d['bench_ok'], round(d['kernel_us'],1), round(d['kernel_us']/$k,1))")"
  done
done
