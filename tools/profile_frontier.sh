#!/bin/bash
# rocprofv3 of the frontier engine's compaction pass (k_level_step) on one MI355X, from the repo root
# on the GPU box: a kernel trace, then FETCH_SIZE and WRITE_SIZE in passes of their own, each over
# tools/bench_frontier.py (cosh4 at eps 1e-12: 25 levels, widest 1.65 M records). Summary:
#   python tools/profile_frontier.py gpurun_out/prof_frontier
set -euo pipefail
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_frontier
mkdir -p "$OUT"
W=${1:-cosh12}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- \
    python3 "$ROOT/tools/bench_frontier.py" --workload "$W" --reps 3 > "$OUT/bench_kt.json" 2> "$OUT/kt.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch_size" -o run -- \
    python3 "$ROOT/tools/bench_frontier.py" --workload "$W" --reps 3 > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write_size" -o run -- \
    python3 "$ROOT/tools/bench_frontier.py" --workload "$W" --reps 3 > "$OUT/bench_write.json" 2> "$OUT/write.err"
