#!/bin/bash
# r06p: C3's host phases without a profiler (AQ_BATCH_TRACE=1): fresh output arrays per call, reused
# output arrays, and one host thread
set -u
OUT=gpurun_out/r06p; mkdir -p $OUT
for v in fresh reuse thr1; do
  args=""; envs="AQ_BATCH_TRACE=1"
  [ $v = reuse ] && args="--reuse-out"
  [ $v = thr1 ] && envs="$envs AQ_HOST_THREADS=1"
  env $envs timeout -k 10 120 python tools/c3_timeline.py --reps 3 $args > $OUT/$v.json 2> $OUT/$v.err || { tail -5 $OUT/$v.err; exit 1; }
  echo "$v $(python3 -c "import json; d=json.load(open('$OUT/$v.json')); print(' '.join('%.3f/%.3f' % (x['wall_ms'], x['kernel_ms']) for x in d['reps']))")"
  grep "aq_integrate_batch n=1000000" $OUT/$v.err | tail -1
done
