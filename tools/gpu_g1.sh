set -o pipefail
mkdir -p gpurun_out/g1
timeout -k 10 60 ./tools/ubench_eval > gpurun_out/g1/ubench.txt 2>&1 || exit 1
timeout -k 10 120 python tools/diag_persist.py --eps 1e-10 --k 256 --reps 3 > gpurun_out/g1/diag256.json 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/g1/counters.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/g1/pmc1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-single --steps 512 --warmup 256 > $GRAFT_REPO_ROOT/gpurun_out/g1/pmc1.out 2>&1
echo pmc1 rc=$?
