#!/bin/bash
# SQ counters of the persistent kernel on the bench launch shape (8192 integrals of cosh4 at
# eps=1e-10 per launch), three rocprofv3 --pmc passes (each within the per-block counter limits),
# from the repo root on the GPU box. Summarise with: python tools/pmc_summary.py gpurun_out/<tag>
set -u
OUT=$PWD/gpurun_out/${1:-pmc}
mkdir -p "$OUT"
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_INSTS_SMEM"
P2="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_BRANCH"
P3="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- python3 "$ROOT/tools/try_kernel.py" --reps 2 --k ${K:-8192} --single 0 --c3 0 > "$OUT/p$i.out" 2>&1 || { echo "pass $i failed"; exit 1; }
done
cd "$ROOT" && python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.json" && cat "$OUT/summary.json"
