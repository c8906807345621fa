#!/bin/bash
# One GPU session of several measurements, each under its own time limit; a failing step ends the
# script (no later GPU step runs after a fault). Output under gpurun_out/<tag>/.
#   tools/gpu_session.sh <tag> [steps...]   steps: tests ubench ab front bench12 bench lone lonecoop shared2 diag smoke ...
#   (AB_GLOB_K / AB_GLOB_F: the library variants the k_stream / frontier A/Bs take)
set -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {   # name seconds command...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  tail -4 "$OUT/$name.out"
  if [ $rc -ne 0 ]; then echo "!! $name rc=$rc"; tail -20 "$OUT/$name.err"; exit $rc; fi
}
for step in "$@"; do
  case $step in
    tests)   run gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    ubench)  run ubench_launch 60 tools/ubench_launch && run ubench_step 120 tools/ubench_step && run ubench_step2 180 tools/ubench_step2 ;;
    ab)      ROUNDS=${ROUNDS:-3} AB_GLOB=${AB_GLOB_K:-libaquad_*.so} run ab 900 bash tools/ab.sh "$TAG" ;;
    front)   AB_GLOB=${AB_GLOB_F:-libaquad_*.so} run front 900 bash tools/frontier_ab.sh "$TAG" ;;
    bench)   run bench 400 python bench.py ;;
    bench12) run bench12 400 python bench.py --eps 1e-12 --batch 4096 --steps 4 --warmup 1 --no-cpu-baseline ;;
    lone)    run lone 120 python tools/try_single.py ;;
    wall)    run wall 120 python tools/try_wall.py ;;
    tiny)    run tiny 120 python tools/try_tiny.py ;;
    tinyvar) for so in ppls_amd/_build/${AB_GLOB_T:-libaquad_*.so}; do n=$(basename $so .so); AQ_LIB=$PWD/$so run tiny_$n 120 python tools/try_tiny.py; done ;;
    lonecoop) AQ_COOP=1 run lone_coop 120 python tools/try_single.py ;;
    shared2) BENCH_SHARED_GPU=1 run shared2 400 python bench.py --gpus 2 --steps 4 --warmup 1 --c3-n 131072 ;;
    diag)    run diag_1e10 120 python tools/diag_single.py --eps 1e-10 && run diag_1task 120 python tools/diag_single.py --eps 1e30 ;;
    smoke)   run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    xcd)     run xcd_start 120 python tools/xcd_start.py ;;
    ulevel)  run ubench_level 120 tools/ubench_level ;;
    stamps)  for so in ppls_amd/_build/libaquad_stamps*.so; do n=$(basename $so .so); AQ_LIB=$PWD/$so run ${n#libaquad_} 120 python tools/stamps_single.py; done ;;
    icache)  run ubench_icache 120 tools/ubench_icache "$OUT/ubench_icache.jsonl" ;;
    pmc)     run pmc 500 bash tools/pmc_profile.sh "pmc_$TAG" ;;
    tests_t) AQ_LIB=$PWD/ppls_amd/_build/libaquad_t_tuned.so run gpu_tests_tuned 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    tests_v) AQ_LIB=$PWD/ppls_amd/_build/${TEST_LIB:?} run gpu_tests_${TEST_LIB%.so} 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    bench_t) AQ_LIB=$PWD/ppls_amd/_build/libaquad_t_tuned.so run bench_tuned 400 python bench.py ;;
    bench12_t) AQ_LIB=$PWD/ppls_amd/_build/libaquad_t_tuned.so run bench12_tuned 400 python bench.py --eps 1e-12 --batch 4096 --steps 4 --warmup 1 --no-cpu-baseline ;;
    prof_t)  AQ_LIB=$PWD/ppls_amd/_build/libaquad_t_tuned.so run prof_tuned 1000 bash tools/profile_round.sh "${TAG}t" ;;
    diagk)   run diag_k32768 300 python tools/diag_persist.py --k 32768 --reps 2 ;;
    lonevar) for so in ppls_amd/_build/${AB_GLOB_L:-libaquad_*.so}; do n=$(basename $so .so); AQ_LIB=$PWD/$so run lone_$n 120 python tools/try_single.py --reps 20; done ;;
    lonesplit) for g in 1 2 3 4; do AQ_GSPLIT=$g run lone_gsplit$g 120 python tools/try_single.py --reps 20; done ;;
    prof)    run prof 1000 bash tools/profile_round.sh "$TAG" ;;
    pmclds)  run pmclds 300 bash tools/pmc_lds.sh "pmc_lds_$TAG" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done ($(date +%T))"
