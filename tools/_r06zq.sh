#!/bin/bash
# r06zq: launches of ~W .. 5W small trees (cosh4 [0,5] at eps=1e-3 / 1e-6): the adaptive default against
# pinned shares per integral (AQ_GSPLIT = waves per share: 1024 -> 3 shares, 512 -> 6)
set -u
OUT=gpurun_out/r06zq; mkdir -p $OUT
for eps in 1e-3 1e-6; do
  for k in 3072 4096 8192 16384; do
    line="eps=$eps k=$k"
    for g in default 1024 512; do
      if [ $g = default ]; then envs=""; else envs="AQ_GSPLIT=$g"; fi
      env $envs timeout -k 10 120 python tools/try_kernel.py --k $k --eps $eps --reps 3 --single 0 --c3 0 > $OUT/$eps.$k.$g.json 2> $OUT/$eps.$k.$g.err || { tail -3 $OUT/$eps.$k.$g.err; exit 1; }
      line="$line | $g $(python3 -c "import json;d=json.load(open('$OUT/$eps.$k.$g.json'));print(d['bench_ok'], round(d['kernel_us'],1))")"
    done
    echo "$line"
  done
done
