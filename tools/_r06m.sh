#!/bin/bash
# r06m: synchronous calls wait on k_fetch_sync's sequence word in pinned memory instead of a stream
# synchronisation (AQ_SYNC_SPIN): GPU suite, then the wall latency A/B (3 alternating passes).
set -u
TAG=r06m
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  for n in libaquad_nospin libaquad; do
    AQ_LIB=$PWD/ppls_amd/_build/$n.so timeout -k 10 120 python tools/try_wall.py > "$OUT/wall_$n.$r.json" 2>&1 || exit 1
    echo "$r $n wall $(cat $OUT/wall_$n.$r.json)"
  done
done
