#!/bin/bash
# Kernel-trace A/B of library variants over the frontier engine (bench_frontier.py cosh12), repo root
# on the GPU box: every ppls_amd/_build/${AB_GLOB:-libaquad_*.so}, then per-level durations via profile_frontier.py
#   tools/frontier_ab.sh <tag>   -> gpurun_out/front_ab_<tag>/<variant>/{bench.json, levels.json}
set -uo pipefail
TAG=${1:?tag}
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
for so in $ROOT/ppls_amd/_build/${AB_GLOB:-libaquad_*.so}; do
  v=$(basename "$so" .so)
  D=$ROOT/gpurun_out/front_ab_$TAG/$v
  mkdir -p $D
  AQ_LIB=$so timeout -k 10 200 python3 $ROOT/tools/bench_frontier.py --workload cosh12 --reps 10 > $D/bench.json 2> $D/err.txt || { tail -5 $D/err.txt; exit 1; }
  AQ_LIB=$so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $D/kt -o run -- python3 $ROOT/tools/bench_frontier.py --workload cosh12 --reps 3 > /dev/null 2>> $D/err.txt || exit 1
  (cd $ROOT && python3 tools/profile_frontier.py $D > $D/levels.json) || true
  echo "$v $(python3 -c "import json;d=json.load(open('$D/bench.json'));print(d['best_ms'],d['median_ms'],d['verified'])") widest $(python3 -c "import json;d=json.load(open('$D/levels.json'));w=d['widest_level'];print(w['us'],w['alg_GBps'],d['sum_level_us'])" 2>/dev/null)"
done
