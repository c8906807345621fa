#!/bin/bash
# r06zm: the batch's first copy + pre-pass and last copy back in order on the launch stream -- GPU suite,
# C3 eps=1e-3 A/B against HEAD (libaquad_hb), host phases of the new code
set -u
OUT=gpurun_out/r06zm; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc -ne 0 ] && exit $rc
ROUNDS=3 SINGLE=0 LIBS="libaquad_hb libaquad" bash tools/ab_c3.sh r06zm > "$OUT/ab_c3.txt" 2>&1 || { tail -5 "$OUT/ab_c3.txt"; exit 1; }
cat "$OUT/ab_c3.txt"
AQ_BATCH_TRACE=1 timeout -k 10 120 python tools/c3_timeline.py --reps 4 > $OUT/trace.json 2> $OUT/trace.err || { tail -5 $OUT/trace.err; exit 1; }
grep "aq_integrate_batch n=1000000" $OUT/trace.err | tail -1
