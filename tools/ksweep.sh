set -o pipefail
mkdir -p gpurun_out/ksweep
for k in 4096 8192 16384 32768; do
  timeout -k 10 200 python tools/try_kernel.py --k $k --reps 2 --single 0 --c3 0 > gpurun_out/ksweep/k$k.json 2>gpurun_out/ksweep/k$k.err || exit 1
  echo "$k $(python3 -c "import json;d=json.load(open('gpurun_out/ksweep/k$k.json'));print(d['bench_ok'], round(d['kernel_us']), '%.4e'%d['accepted_per_s_kernel'])")"
done
