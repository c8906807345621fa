#!/bin/bash
# r06w: sin(1/x) batches of 4096 (the bench's C4 pass shape) against the job size -- the adaptive hint
# (default) and AQ_GSPLIT = waves per job pinned (3072 waves: 1 / 3 / 6 / 12 / 24 shares per integral)
set -u
OUT=gpurun_out/r06w; mkdir -p $OUT
for r in 1 2; do
  for g in default 3072 1024 512 256 128; do
    if [ $g = default ]; then
      timeout -k 10 120 python tools/try_sin_batch.py --k 64,4096 --reps 5 > $OUT/g$g.$r.json 2>&1 || { tail -3 $OUT/g$g.$r.json; exit 1; }
    else
      AQ_GSPLIT=$g timeout -k 10 120 python tools/try_sin_batch.py --k 64,4096 --reps 5 > $OUT/g$g.$r.json 2>&1 || { tail -3 $OUT/g$g.$r.json; exit 1; }
    fi
    echo "$r gsplit=$g $(tail -1 $OUT/g$g.$r.json)"
  done
done
