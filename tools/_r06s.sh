#!/bin/bash
# r06s: C3 at eps=1e-10 -- wall against kernel per call (host phases on), the DIAG instance on one
# 262144-integral C3 launch against the bench's 32768 x [0,5] launch
set -u
OUT=gpurun_out/r06s; mkdir -p $OUT
AQ_BATCH_TRACE=1 timeout -k 10 200 python tools/c3_timeline.py --eps 1e-10 --reps 2 > $OUT/c3_1e10.json 2> $OUT/c3_1e10.err || { tail -5 $OUT/c3_1e10.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/c3_1e10.json')); print(' '.join('%.3f/%.3f/%d' % (x['wall_ms'], x['kernel_ms'], x['launches']) for x in d['reps']))"
grep "aq_integrate_batch n=1000000" $OUT/c3_1e10.err | tail -1
timeout -k 10 200 python tools/diag_persist.py --k 262144 --eps 1e-10 --c3 --reps 1 --out $OUT/diag_c3_1e10.json > $OUT/diag_c3_1e10.out 2>&1 || { tail -5 $OUT/diag_c3_1e10.out; exit 1; }
timeout -k 10 200 python tools/diag_persist.py --k 32768 --eps 1e-10 --reps 1 --out $OUT/diag_bench.json > $OUT/diag_bench.out 2>&1 || { tail -5 $OUT/diag_bench.out; exit 1; }
python3 - <<'PY'
import json
for f in ('gpurun_out/r06s/diag_c3_1e10.json', 'gpurun_out/r06s/diag_bench.json'):
    s = json.load(open(f))['summaries'][-1]
    print(f, {k: s[k] for k in ('lanes_per_round', 'tasks_per_round', 'share_of_loop', 'cyc_per_round', 'cyc_seed_per_call')}, s['seed_calls'], s['t_exit'], s['t_first_lead'])
PY
