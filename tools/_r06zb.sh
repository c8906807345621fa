#!/bin/bash
# r06zb: cosh4 eps=1e-12 x 256 (and 64) repeated, alternating libaquad_hb / libaquad (variance check)
set -u
OUT=gpurun_out/r06zb; mkdir -p $OUT
for r in 1 2 3 4; do
  for k in 256 64; do
    line="pass $r k=$k"
    for n in libaquad_hb libaquad; do
      AQ_LIB=$PWD/ppls_amd/_build/$n.so timeout -k 10 120 python tools/try_kernel.py --k $k --eps 1e-12 --reps 3 --single 0 --c3 0 > $OUT/$n.$k.$r.json 2> $OUT/$n.$k.$r.err || { tail -3 $OUT/$n.$k.$r.err; exit 1; }
      line="$line | $n $(python3 -c "import json;d=json.load(open('$OUT/$n.$k.$r.json'));print(d['bench_ok'], round(d['kernel_us'],1))")"
    done
    echo "$line"
  done
done
