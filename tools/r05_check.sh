#!/bin/bash
# GPU tests, then the C3 pass's device timeline and the bench line (run on the GPU box from the repo root).
# Usage: tools/r05_check.sh <tag> [notests] [nobench]
set -u
TAG=${1:?tag}; shift
ROOT=$PWD
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
if [[ " $* " != *" notests "* ]]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
  rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc -ne 0 ] && exit $rc
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/c3tl" -o run -- \
    python3 "$ROOT/tools/c3_timeline.py" > "$OUT/c3tl.out" 2>&1 || { echo "c3 timeline failed"; exit 1; }
grep '^{' "$OUT/c3tl.out"
cd "$ROOT"
if [[ " $* " != *" nobench "* ]]; then
  timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -5 "$OUT/bench.err"; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/bench.json'))
print('value', d['value'], 'frac', d['roofline']['frac'], 'single_us', d['single_integral_kernel_us'], 'verified', d['verified'])
for s in d['secondary']: print(s['workload'][:40], 'ms', round(s['ms'],3), 'frac', s['frac'], s['verified'])
"
fi
find "$OUT" -type f -size +4M -print -delete
echo done
