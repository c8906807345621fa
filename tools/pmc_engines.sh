#!/bin/bash
# SQ counters of the persistent kernels (one rocprofv3 --pmc pass per engine), from the repo root on the GPU box.
set -u
OUT=$PWD/gpurun_out/${1:-pmc}
mkdir -p "$OUT"
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp
for eng in ${ENGINES:-stream dfs}; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY \
     --output-format csv -d "$OUT/$eng" -o run -- python3 "$ROOT/tools/try_engine.py" --engine $eng --reps 2 > "$OUT/$eng.out" 2>&1 || exit 1
done
cd "$ROOT"
python3 tools/pmc_summary.py "$OUT"
