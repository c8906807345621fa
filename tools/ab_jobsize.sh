set -o pipefail
mkdir -p gpurun_out/tpj
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tpj/gpu_tests.log 2>&1 || exit 1
for l in libaquad libaquad_tpj15000; do
  AQ_LIB=$PWD/ppls_amd/_build/$l.so timeout -k 10 200 python tools/bench_batch.py --reps 2 > gpurun_out/tpj/batch_$l.json 2>/dev/null || exit 1
  AQ_LIB=$PWD/ppls_amd/_build/$l.so timeout -k 10 200 python bench.py --eps 1e-12 --no-cpu-baseline --no-single > gpurun_out/tpj/b12_$l.json 2>/dev/null || exit 1
done
for l in libaquad libaquad_gs64 libaquad_gs96; do
  AQ_LIB=$PWD/ppls_amd/_build/$l.so BENCH_SHARED_GPU=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29551 bench.py --gpus 2 --no-single > gpurun_out/tpj/n2_$l.json 2> gpurun_out/tpj/n2_$l.err || exit 1
done
