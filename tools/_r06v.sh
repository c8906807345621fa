#!/bin/bash
# r06v: where a synchronous call's wall goes -- HIP runtime API + kernel trace of tools/try_wall.py
set -u
OUT=$PWD/gpurun_out/r06v; ROOT=$PWD; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --runtime-trace --kernel-trace --output-format csv -d "$OUT/rt" -o run -- \
    python3 "$ROOT/tools/try_wall.py" --reps 20 > "$OUT/rt.out" 2>&1 || { echo "trace failed"; tail -5 $OUT/rt.out; exit 1; }
cd $ROOT
cat $OUT/rt.out | tail -2
timeout -k 10 120 python tools/try_wall.py --reps 200 > $OUT/wall.json 2>&1 || exit 1
cat $OUT/wall.json
find $OUT -name "*.csv" -size +4M -print -delete
