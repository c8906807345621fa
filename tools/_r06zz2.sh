#!/bin/bash
# r06zz2: synchronous waits hand over to the stream synchronisation past 2 ms -- GPU suite, wall of
# short synchronous calls, and one long one (eps=1e-16, ~150 M tasks) against the reference's count
set -u
OUT=gpurun_out/r06zz2; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/try_wall.py --reps 100 > $OUT/wall.json 2>&1 || exit 1
cat $OUT/wall.json
timeout -k 10 120 python - <<'PY'
import json, time
from ppls_amd import Context, Problem
g = json.load(open("tests/golden/deep.json"))["cosh4_eps1e-16"]
with Context(0) as c:
    c.set_level_histograms(False)
    t0 = time.perf_counter(); r = c.integrate(Problem(eps=1e-16)); t1 = time.perf_counter()
    print("eps1e-16 sync", round((t1 - t0) * 1e3, 2), "ms", r.tasks, r.tasks == g["tasks"])
PY
