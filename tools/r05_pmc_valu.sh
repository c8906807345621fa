#!/bin/bash
# FP64 / VALU counters of the bench's persistent launch (run on the GPU box from the repo root):
# a kernel-trace pass and four SQ / GRBM --pmc passes (each within the per-block counter limits) of
# tools/pmc_bench_launch.py (32768 x cosh4 [0,5] at eps=1e-10 per launch), the DIAG instance's
# lanes per round on the same launch, then tools/pmc_valu.py folds them into pmc_valu.json.
# Raw CSVs above 4 MiB are dropped so the merge-back stays small.
# Usage: tools/r05_pmc_valu.sh <tag> [extra args for pmc_bench_launch.py]
set -u
TAG=${1:-r05b}; shift
ROOT=$PWD
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
CMD=(python3 "$ROOT/tools/pmc_bench_launch.py" "$@")
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- "${CMD[@]}" \
    > "$OUT/kt.out" 2>&1 || { echo "kernel trace failed"; exit 1; }
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_INSTS_SMEM"
P2="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_BRANCH"
P3="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA"
P4="GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- "${CMD[@]}" \
      > "$OUT/p$i.out" 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
cd "$ROOT"
timeout -k 10 120 python3 tools/diag_persist.py --k 32768 --eps 1e-10 --reps 1 --out "$OUT/diag_bench.json" \
    > "$OUT/diag_bench.out" 2>&1 || { echo "diag bench failed"; exit 1; }
TPR=$(python3 -c "import json; print(json.load(open('$OUT/diag_bench.json'))['summaries'][-1]['tasks_per_round'])")
python3 tools/pmc_valu.py "$OUT" --tasks-per-round "$TPR" --tag "$TAG" > "$OUT/pmc_valu.json" || { echo "summary failed"; exit 1; }
cat "$OUT/pmc_valu.json"
find "$OUT" -type f -size +4M -print -delete
echo done
