set -euo pipefail
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
for v in lr2 lr4 lr8; do
  mkdir -p $ROOT/gpurun_out/front_ab/$v
  AQ_LIB=$ROOT/ppls_amd/_build/libaquad_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $ROOT/gpurun_out/front_ab/$v/kt -o run -- python3 $ROOT/tools/bench_frontier.py --workload cosh12 --reps 3 > $ROOT/gpurun_out/front_ab/$v/bench.json 2> $ROOT/gpurun_out/front_ab/$v/err.txt
done
