#!/bin/bash
# r06zz: lone integrals of deep trees (eps 1e-13 .. 1e-15) -- the 8-wave lone instance against 12 waves
set -u
OUT=gpurun_out/r06zz; mkdir -p $OUT
for r in 1 2; do
  for n in libaquad libaquad_nw12; do
    AQ_LIB=$PWD/ppls_amd/_build/$n.so timeout -k 10 200 python tools/try_single.py --reps 20 --deep > $OUT/$n.$r.json 2> $OUT/$n.$r.err || { tail -3 $OUT/$n.$r.err; exit 1; }
    echo "$r $n $(cat $OUT/$n.$r.json)"
  done
done
