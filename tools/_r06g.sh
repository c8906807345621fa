#!/bin/bash
# r06g: level-step prefetch (resident grid, next chunk in flight) -- GPU suite on the new default, then
# the frontier engine's per-level kernel trace for: r05 behavior (lvbase), prefetch R=4 (lvpf4), R=2 (lvpf2)
set -u
OUT=gpurun_out/r06g; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  AB_GLOB="libaquad_lv*.so" timeout -k 10 900 bash tools/frontier_ab.sh r06g_$r > $OUT/front_ab_$r.txt 2>&1 || { tail -5 $OUT/front_ab_$r.txt; exit 1; }
  cat $OUT/front_ab_$r.txt
done
