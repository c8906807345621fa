#!/bin/bash
# LDS-side counters of the persistent kernel on the tools/try_kernel.py bench shape (8192 integrals of
# cosh4 at eps=1e-10 per launch): is the CU's LDS (array cycles, bank conflicts, instruction issue
# waits) a co-bottleneck beside the VALU? One rocprofv3 --pmc pass per counter group, from the repo
# root on the GPU box; the counter list of the device goes to gpurun_out/<tag>/counters.txt.
set -u
OUT=$PWD/gpurun_out/${1:-pmc_lds}
mkdir -p "$OUT"
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
P1="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU"
i=0
for P in "$P1"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- python3 "$ROOT/tools/try_kernel.py" --reps 2 --k ${K:-8192} --single 0 --c3 0 > "$OUT/p$i.out" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.out"; exit 1; }
done
cd "$ROOT" && python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.json" && cat "$OUT/summary.json"
