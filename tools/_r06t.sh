#!/bin/bash
# r06t: where C3 eps=1e-10 loses against the bench launch -- AQ_STAMPS timelines of a size-ordered
# 262144-integral C3 launch (the last of a 393216-integral batch) and of the bench's 32768 x [0,5] launch
set -u
OUT=gpurun_out/r06t; mkdir -p $OUT
L=$PWD/ppls_amd/_build/libaquad_stamps.so
AQ_LIB=$L timeout -k 10 300 python tools/stamps_burst.py --k 393216 --eps 1e-10 --c3 --batch > $OUT/burst_c3_1e10.json 2> $OUT/c3.err || { tail -5 $OUT/c3.err; exit 1; }
cat $OUT/burst_c3_1e10.json
AQ_LIB=$L timeout -k 10 300 python tools/stamps_burst.py --k 32768 --eps 1e-10 > $OUT/burst_bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cat $OUT/burst_bench.json
