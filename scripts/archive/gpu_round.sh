#!/bin/bash
# One GPU session: parity tests, smoke, bench lines, rocprofv3 kernel-trace summary.
# Each GPU step has its own time limit; a crash/fault/timeout (rc other than 0/1)
# stops the script so nothing else touches the GPU after a fault.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -5 $OUT/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-"pytest smoke bench_fp32 bench_simd prof pmc"}
for s in $STEPS; do
  case $s in
    pytest) step pytest 1200 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ;;
    bench) step bench 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench_fp32) step bench_fp32 600 python bench.py --mode fp32 --steps 20 --warmup 3 ;;
    bench_simd) step bench_simd 600 python bench.py --mode simd --steps 20 --warmup 3 --cpu-baseline off ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off --host-boundary off ;;
    pmc) step pmc_fp32 900 bash scripts/profile_pmc.sh fp32 &&
         step pmc_simd 900 bash scripts/profile_pmc.sh simd &&
         python scripts/pmc_summary.py $OUT/pmc_fp32 scoreSplit --json $OUT/pmc_fp32.json > /dev/null &&
         python scripts/pmc_summary.py $OUT/pmc_simd scoreI8 --json $OUT/pmc_simd.json > /dev/null ;;
    sweep) step sweep 1200 bash scripts/sweep_batch.sh ;;
    bench_d45) step bench_d45 600 python bench.py --dim 45 --steps 20 --warmup 3 --cpu-baseline off --host-boundary off ;;
    bench_ragged) step bench_ragged 600 python bench.py --ragged --steps 20 --warmup 3 --cpu-baseline off --host-boundary off ;;
    bench_sum) step bench_sum 600 python bench.py --mode sum --steps 20 --warmup 3 --cpu-baseline off --host-boundary off --no-extra-mode ;;
    bench_nn) step bench_nn 600 python bench.py --mode nn --steps 20 --warmup 3 ;;
    bench_presel) step bench_presel_int 600 python bench.py --mode presel-int --steps 10 --warmup 2 --cpu-baseline off --host-boundary off --no-extra-mode &&
                  step bench_presel_float 600 python bench.py --mode presel-float --steps 10 --warmup 2 --cpu-baseline off --host-boundary off --no-extra-mode ;;
    pytest_new) step pytest_new 1200 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $PYTEST_ARGS ;;
  esac
done
echo done
