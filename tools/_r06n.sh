#!/bin/bash
# r06n: the batch's size-order pre-pass on its own stream (chunk c + 1's beside chunk c's gather) --
# GPU suite, C3 eps=1e-3 A/B against the serial pre-pass (libaquad_ser = HEAD before it), and the device
# timeline of one 1 M-integral call of the new code.
set -u
TAG=r06n
OUT=$PWD/gpurun_out/$TAG; ROOT=$PWD
mkdir -p "$OUT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc -ne 0 ] && exit $rc
ROUNDS=3 SINGLE=0 LIBS="libaquad_ser libaquad" bash tools/ab_c3.sh $TAG > "$OUT/ab_c3.txt" 2>&1 || { tail -5 "$OUT/ab_c3.txt"; exit 1; }
cat "$OUT/ab_c3.txt"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/c3tl" -o run -- \
    python3 "$ROOT/tools/c3_timeline.py" > "$OUT/c3tl.out" 2>&1 || { echo "c3 timeline failed"; tail -5 $OUT/c3tl.out; exit 1; }
cd $ROOT
python3 tools/c3_timeline_summary.py $OUT/c3tl --what "r06n pre-pass on s_pre" > $OUT/c3_timeline.json || exit 1
python3 -c "
import json; d=json.load(open('$OUT/c3_timeline.json'))
print(d['calls_seen'], d['span_us'], d['k_stream_cover_us'], d['outside_k_stream_us'])
for e in d['events']: print(e['start_us'], e['dur_us'], e['op'][:40])
"
find "$OUT" -type f -size +4M -print -delete
