#!/bin/bash
# r06r: batch host work on the persistent pool, with and without first-touching each chunk's output
# pages during its kernel, against the code before the pre-pass stream and the pool (libaquad_ser):
# GPU suite, then C3 eps=1e-3 (fresh output arrays per call) in 3 alternating passes
set -u
OUT=gpurun_out/r06r; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc -ne 0 ] && exit $rc
ROUNDS=3 SINGLE=0 LIBS="libaquad_ser libaquad_nopf libaquad" bash tools/ab_c3.sh r06r > "$OUT/ab_c3.txt" 2>&1 || { tail -5 "$OUT/ab_c3.txt"; exit 1; }
cat "$OUT/ab_c3.txt"
AQ_BATCH_TRACE=1 timeout -k 10 120 python tools/c3_timeline.py --reps 4 > $OUT/trace.json 2> $OUT/trace.err || { tail -5 $OUT/trace.err; exit 1; }
grep "aq_integrate_batch n=1000000" $OUT/trace.err | tail -1
