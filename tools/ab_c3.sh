#!/bin/bash
# Alternating A/B of library variants on the C3 batch (tools/c3_timeline.py: 1 M integrals at eps=1e-3
# through aq_integrate_batch, wall and kernel time) and on lone integrals (tools/try_single.py), one
# process per run, ROUNDS passes over ppls_amd/_build/libaquad*.so (run on the GPU box, repo root).
#   tools/ab_c3.sh <tag>   (env: ROUNDS=3 LIBS="libaquad libaquad_x" SINGLE=1 EPS=1e-3)
set -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/ab_$TAG
mkdir -p "$OUT"
LIBS=${LIBS:-$(cd ppls_amd/_build && ls libaquad*.so | sed 's/\.so$//')}
for r in $(seq 1 ${ROUNDS:-3}); do
  for n in $LIBS; do
    so=$PWD/ppls_amd/_build/$n.so
    AQ_LIB=$so timeout -k 10 120 python tools/c3_timeline.py --reps 3 --eps ${EPS:-1e-3} > "$OUT/$n.c3.$r.json" 2> "$OUT/$n.c3.$r.err" \
        || { echo "$n c3 failed"; tail -5 "$OUT/$n.c3.$r.err"; exit 1; }
    echo "$r $n c3 $(python3 -c "import json; d=json.load(open('$OUT/$n.c3.$r.json')); print(' '.join('%.3f/%.3f' % (x['wall_ms'], x['kernel_ms']) for x in d['reps']), all(x['t_eq_2l_1'] for x in d['reps']))")"
    if [ "${SINGLE:-1}" = 1 ]; then
      AQ_LIB=$so timeout -k 10 120 python tools/try_single.py --reps 30 > "$OUT/$n.single.$r.json" 2> "$OUT/$n.single.$r.err" \
          || { echo "$n single failed"; tail -5 "$OUT/$n.single.$r.err"; exit 1; }
      echo "$r $n single $(cat "$OUT/$n.single.$r.json")"
    fi
  done
done
