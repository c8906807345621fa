set -o pipefail
mkdir -p gpurun_out/diag_ab
for v in pipe0 pipe1; do
  AQ_LIB=$PWD/ppls_amd/_build/libaquad_$v.so timeout -k 10 120 python tools/diag_persist.py --k 8192 --reps 2 > gpurun_out/diag_ab/$v.json 2>gpurun_out/diag_ab/$v.err || { tail gpurun_out/diag_ab/$v.err; exit 1; }
done
