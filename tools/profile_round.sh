#!/bin/bash
# Round profile of the bench command on one MI355X (run on the GPU box from the repo root):
#   1. rocprofv3 --kernel-trace --stats        -> per-kernel durations
#   2. rocprofv3 --pmc FETCH_SIZE  (own pass)  -> HBM read bytes per dispatch
#   3. rocprofv3 --pmc WRITE_SIZE  (own pass)  -> HBM write bytes per dispatch
# then tools/profile_summary.py folds them into profiles/<tag>_*.
# Usage: tools/profile_round.sh <tag> [bench args...]
set -euo pipefail
TAG=${1:?tag}; shift
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(--no-cpu-baseline --no-single --no-secondary --steps 8 --warmup 1)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- \
    python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/bench_kt.json" 2> "$OUT/kt.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 "$ROOT/bench.py" "${ARGS[@]}" > "$OUT/bench_write.json" 2> "$OUT/write.err"
cd "$ROOT"
python3 tools/profile_summary.py "$TAG" "$OUT"
