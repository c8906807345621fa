#!/bin/bash
# r06z: the few-integral fill rule on cosh4 [0,5] launches of 16 .. 2048 copies at eps=1e-10 / 1e-8 / 1e-12,
# against the code before it (libaquad_hb); kernel us per launch, counts checked; k = 1024 / 2048 (the
# HEAPS instance now, same shares) in 3 alternating passes
set -u
OUT=gpurun_out/r06z; mkdir -p $OUT
run() {  # lib eps k tag
  AQ_LIB=$PWD/ppls_amd/_build/$1.so timeout -k 10 120 python tools/try_kernel.py --k $3 --eps $2 --reps 3 --single 0 --c3 0 > $OUT/$1.$2.$3.$4.json 2> $OUT/$1.$2.$3.$4.err || { tail -3 $OUT/$1.$2.$3.$4.err; return 1; }
  python3 -c "import json;d=json.load(open('$OUT/$1.$2.$3.$4.json'));print(d['bench_ok'], round(d['kernel_us'],1))"
}
for eps in 1e-10 1e-8 1e-12; do
  for k in 16 64 256; do
    a=$(run libaquad_hb $eps $k 0) || exit 1; b=$(run libaquad $eps $k 0) || exit 1
    echo "eps=$eps k=$k | hb $a | new $b"
  done
done
for r in 1 2 3; do
  for k in 1024 2048; do
    a=$(run libaquad_hb 1e-10 $k $r) || exit 1; b=$(run libaquad 1e-10 $k $r) || exit 1
    echo "pass $r eps=1e-10 k=$k | hb $a | new $b"
  done
done
