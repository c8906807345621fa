#!/bin/bash
# r06f: the bench with the C4 secondary pass (N=1), and the N=2 shared-GPU rehearsal of the bench path
set -u
OUT=gpurun_out/r06f; mkdir -p $OUT
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench.json')); r=d['roofline']
print('value', d['value'], 'ms/step', d['ms_per_step'], 'frac', r['frac'], 'single_us', d.get('single_integral_kernel_us'), 'verified', d['verified'])
for s in d.get('secondary', []): print(s['workload'][:60], 'ms', round(s['ms'], 3), 'frac', s['frac'], s['verified'], s.get('single_integral_kernel_us'))
"
BENCH_SHARED_GPU=1 timeout -k 10 600 python bench.py --gpus 2 --steps 4 --warmup 1 --c3-n 131072 > $OUT/shared2.json 2> $OUT/shared2.err || { tail -5 $OUT/shared2.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/shared2.json'))
print('shared2 ranks', d['ranks_seen'], 'verified', d['verified'], d['checks'], [ (s['workload'][:12], s['verified']) for s in d['secondary']])
"
