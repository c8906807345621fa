#!/bin/bash
# r06k: round-end evidence on the final code -- GPU suite, smoke, the default bench line, then the
# 8-rank shared-GPU rehearsal of the N=8 bench path.
set -u
TAG=${TAG:-r06k}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
bash tools/r05_final.sh $TAG || exit $?
BENCH_SHARED_GPU=1 timeout -k 10 600 python bench.py --gpus 8 --steps 20 --warmup 5 > $OUT/shared8_bench.json 2> $OUT/shared8.err
rc=$?; tail -3 $OUT/shared8.err; [ $rc -ne 0 ] && exit $rc
SHARED8=$OUT/shared8_bench.json python3 - <<'PY'
import json
import os
lines = [l for l in open(os.environ["SHARED8"]) if l.startswith("{")]
d = json.loads(lines[-1])
print(d["value"], d["verified"], d["ranks_seen"], d["per_rank"]["task_imbalance"], [(s["ms"], s["verified"]) for s in d.get("secondary") or []])
PY
