#!/bin/bash
# VALU instruction mix of the persistent kernel (two rocprofv3 --pmc passes), from the repo root on the GPU box.
set -u
OUT=$PWD/gpurun_out/${1:-pmcv}
mkdir -p "$OUT"
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_INSTS_SMEM"
P2="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_BRANCH"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- python3 "$ROOT/tools/try_engine.py" --engine stream --reps 2 --k ${K:-8192} > "$OUT/p$i.out" 2>&1 || echo "pass $i failed"
done
