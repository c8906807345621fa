#!/bin/bash
# Round-end evidence on one MI355X (run on the GPU box from the repo root): the GPU suite, smoke(), the
# default bench line. Usage: tools/r05_final.sh <tag>
set -u
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { tail -5 "$OUT/smoke.txt"; exit 1; }
cat "$OUT/smoke.txt"
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json'))
r=d['roofline']
print('value', d['value'], 'ms/step', d['ms_per_step'], 'frac', r['frac'], 'issue', r.get('issue_bound'), 'single_us', d.get('single_integral_kernel_us'), 'verified', d['verified'])
for s in d.get('secondary', []): print(s['workload'][:50], 'ms', round(s['ms'], 3), 'frac', s['frac'], s['verified'])
"
