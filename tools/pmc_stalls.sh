#!/bin/bash
# Stall / LDS counters of the persistent kernel (two rocprofv3 --pmc passes), from the repo root on the GPU box.
set -u
OUT=$PWD/gpurun_out/${1:-pmcs}
mkdir -p "$OUT"
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_THREAD_CYCLES_VALU"
P2="SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS SQ_BUSY_CYCLES SQ_LDS_ADDR_CONFLICT"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- python3 "$ROOT/tools/try_engine.py" --engine stream --reps 2 --k 2048 > "$OUT/p$i.out" 2>&1 || echo "pass $i failed"
done
