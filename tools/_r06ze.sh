#!/bin/bash
# r06ze: unsharded launches of 12-15 integrals claim filled jobs -- GPU suite, then the small-launch sweep
set -u
OUT=gpurun_out/r06ze; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc -ne 0 ] && exit $rc
sed 's#gpurun_out/r06zd#gpurun_out/r06ze#' tools/_r06zd.sh > /tmp/zd.sh && bash /tmp/zd.sh
