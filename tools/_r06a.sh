#!/bin/bash
# r06a: round-6 baseline on a fresh box -- GPU suite, smoke, bench, and a kernel trace WITH timestamps
# of the headline launches (the gaps between k_stream dispatches: ms_per_step - kernel time).
set -u
TAG=r06a
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
bash tools/r05_final.sh $TAG || exit $?
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/$OUT/kt" -o run -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --no-single --no-secondary --steps 8 --warmup 1 \
    > "$ROOT/$OUT/bench_kt.json" 2> "$ROOT/$OUT/kt.err" || { tail -5 "$ROOT/$OUT/kt.err"; exit 1; }
cd "$ROOT"
find "$OUT/kt" -name "*kernel_trace.csv" | head -3
