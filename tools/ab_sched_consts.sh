#!/bin/bash
# A/B the stream farmer's scheduling constants (POLL_ROUNDS, GIVE_ROUNDS, GIVE_MIN) on one box:
# bench.py (eps 1e-10, 8192 integrals per launch) against each ppls_amd/_build/libaquad*.so,
# two interleaved passes so drift shows. Run from the repo root on the GPU box.
set -o pipefail
mkdir -p gpurun_out/abc
for rep in 1 2; do
  for so in ppls_amd/_build/libaquad*.so; do
    n=$(basename $so .so)
    AQ_LIB=$PWD/$so timeout -k 10 120 python bench.py --no-cpu-baseline --no-single --steps 8 --warmup 2 \
      > gpurun_out/abc/${n}_$rep.json 2> gpurun_out/abc/${n}_$rep.err || { echo "$n failed"; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/abc/${n}_$rep.json'));r=d['roofline'];print('$n rep$rep', d['verified'], round(r['kernel_avg_us'],1), '%.4e'%d['value'])" | tee -a gpurun_out/abc/summary.txt
    if [ $rep = 1 ]; then
      AQ_LIB=$PWD/$so timeout -k 10 120 python tools/try_engine.py --engine stream --reps 3 --k 1 \
        > gpurun_out/abc/${n}_single.json 2>&1 || { echo "$n single failed"; exit 1; }
      AQ_LIB=$PWD/$so timeout -k 10 200 python tools/bench_batch.py --reps 2 \
        > gpurun_out/abc/${n}_c3.json 2> gpurun_out/abc/${n}_c3.err || { echo "$n c3 failed"; exit 1; }
    fi
  done
done
