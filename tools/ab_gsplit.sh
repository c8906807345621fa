mkdir -p gpurun_out/gs
for g in ${GSPLITS:-0 16 32 64}; do
  AQ_GSPLIT=$g timeout -k 10 120 python tools/try_engine.py --engine stream --reps ${REPS:-3} --k ${K:-2048} > gpurun_out/gs/$g.json 2>&1 || { echo "$g failed"; exit 1; }
  echo "gsplit $g $(python3 -c "import json;d=json.load(open('gpurun_out/gs/$g.json'));print(d['bench_ok'], round(d['kernel_us'],1), '%.3e'%d['accepted_per_s_kernel'])")"
done
