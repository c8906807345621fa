#!/bin/bash
# r06zg: round-end evidence on HEAD (GPU suite, smoke, bench, 8-rank rehearsal), then the small-launch
# sweeps on the final code
set -u
TAG=r06zg bash tools/_r06k.sh || exit $?
sed 's#gpurun_out/r06zd#gpurun_out/r06zg#' tools/_r06zd.sh > /tmp/zd.sh && bash /tmp/zd.sh || exit 1
timeout -k 10 200 python tools/try_sin_batch.py --k 1,2,4,8,11,12,16,64,4096 --reps 5 > gpurun_out/r06zg/sin.json 2>&1 || { tail -3 gpurun_out/r06zg/sin.json; exit 1; }
tail -1 gpurun_out/r06zg/sin.json
