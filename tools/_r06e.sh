#!/bin/bash
# r06e: stamps of the current code -- lone-integral timeline (8-wave instance, PCU_AREA exit) and where a
# C3 eps=1e-3 batch launch's wave time goes (heap seeding of whole-integral jobs)
set -u
OUT=gpurun_out/r06e; mkdir -p $OUT
L=$PWD/ppls_amd/_build/libaquad_stamps.so
AQ_LIB=$L timeout -k 10 120 python tools/stamps_single.py > $OUT/stamps8.json 2> $OUT/stamps8.err || { tail -5 $OUT/stamps8.err; exit 1; }
AQ_LIB=$L timeout -k 10 120 python tools/stamps_burst.py --k 393216 --eps 1e-3 --c3 --batch > $OUT/burst_c3_batch.json 2> $OUT/burst_c3.err || { tail -5 $OUT/burst_c3.err; exit 1; }
AQ_LIB=$L timeout -k 10 180 python tools/stamps_burst.py --k 32768 --eps 1e-10 > $OUT/burst_bench.json 2> $OUT/burst_bench.err || { tail -5 $OUT/burst_bench.err; exit 1; }
cat $OUT/burst_c3_batch.json; echo; cat $OUT/burst_bench.json
python3 - <<'PY'
import json
d=json.load(open('gpurun_out/r06e/stamps8.json'))
for k,v in d.items():
  if isinstance(v,dict) and 'kernel_us' in v:
    print(k, v['kernel_us'], {p: v[p][1:4] for p in d['points'] if p in v})
PY
