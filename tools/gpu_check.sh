#!/bin/bash
# One GPU check pass (repo root, on the GPU box): pytest -m gpu, then optional steps by flag:
#   tools/gpu_check.sh <tag> [bench] [frontier] [bench12]
# -> gpurun_out/<tag>/{gpu_tests.log, bench.json, bench12.json, frontier_*.json, frontier_levels.json}
set -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?
tail -3 "$OUT/gpu_tests.log"
[ $rc -ne 0 ] && exit $rc
for step in "$@"; do
  case $step in
    bench) timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1 ;;
    bench12) timeout -k 10 400 python bench.py --eps 1e-12 --steps 4 --no-cpu-baseline > "$OUT/bench12.json" 2> "$OUT/bench12.err" || exit 1 ;;
    frontier)
      for w in cosh12 cosh10 sin; do
        timeout -k 10 120 python tools/bench_frontier.py --workload $w --reps 10 > "$OUT/frontier_$w.json" || exit 1
      done
      bash tools/profile_frontier.sh cosh12 && python tools/profile_frontier.py gpurun_out/prof_frontier > "$OUT/frontier_levels.json" ;;
  esac
done
