#!/bin/bash
# Instruction-fetch counters of lone-integral launches (tools/try_single.py shapes), two rocprofv3
# --pmc passes (SQC block, SQ block), from the repo root on the GPU box. Diagnostic tool.
#   bash tools/pmc_icache.sh <tag>   ->  gpurun_out/<tag>/{c1,c2}/run_counter_collection.csv
set -u
OUT=$PWD/gpurun_out/${1:-icache}
mkdir -p "$OUT"
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp
P1="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"
P2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAIT_ANY"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d "$OUT/c$i" -o run -- python3 "$ROOT/tools/try_single.py" --reps 5 > "$OUT/c$i.out" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/c$i.out"; exit 1; }
done
