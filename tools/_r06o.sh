#!/bin/bash
# r06o: where C3's wall outside the device span goes -- HIP runtime API trace + kernel + copy trace of
# tools/c3_timeline.py (1 M integrals at eps=1e-3, two timed calls)
set -u
OUT=$PWD/gpurun_out/r06o; ROOT=$PWD; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --runtime-trace --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/rt" -o run -- \
    python3 "$ROOT/tools/c3_timeline.py" --reps 2 > "$OUT/rt.out" 2>&1 || { echo "trace failed"; tail -5 $OUT/rt.out; exit 1; }
cd $ROOT
grep '^{' $OUT/rt.out
find $OUT -name "*.csv" -exec ls -la {} \;
