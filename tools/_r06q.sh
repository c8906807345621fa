#!/bin/bash
# r06q: the batch's host work on a persistent thread pool -- GPU suite, then C3's host phases
# (AQ_BATCH_TRACE=1) with fresh and reused output arrays and with one host thread
set -u
OUT=gpurun_out/r06q; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc -ne 0 ] && exit $rc
for v in fresh reuse thr1 fresh2 reuse2; do
  args=""; envs="AQ_BATCH_TRACE=1"
  case $v in reuse*) args="--reuse-out";; thr1) envs="$envs AQ_HOST_THREADS=1";; esac
  env $envs timeout -k 10 120 python tools/c3_timeline.py --reps 4 $args > $OUT/$v.json 2> $OUT/$v.err || { tail -5 $OUT/$v.err; exit 1; }
  echo "$v $(python3 -c "import json; d=json.load(open('$OUT/$v.json')); print(' '.join('%.3f/%.3f' % (x['wall_ms'], x['kernel_ms']) for x in d['reps']))")"
  grep "aq_integrate_batch n=1000000" $OUT/$v.err | tail -1
done
