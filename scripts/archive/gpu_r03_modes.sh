#!/bin/bash
# Round-3: the other bench lines on the HEAD build (diagonal-sum, preselection int / float, hybrid DNN, config 3's
# D = 45, the ragged model), each with its rocprofv3 kernel-trace summary; plus the sharded-scorer GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN:-r03_modes}
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -2 $OUT/$name.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step sharded_tests 400 python -u -m pytest tests/test_sharded_scorer.py -q -m gpu --timeout 120 --timeout-method thread
B="--gpus 1 --steps 20 --warmup 3 --cpu-baseline off --host-boundary off --extras off --no-extra-mode"
step bench_sum 300 python bench.py --mode sum $B
step bench_sum_scores 300 python bench.py --mode sum --no-best $B
step bench_d45_simd_scores 300 python bench.py --dim 45 --mode simd-scores $B
step bench_presel_int 300 python bench.py --mode presel-int $B
step bench_presel_float 300 python bench.py --mode presel-float $B
step bench_nn 300 python bench.py --mode nn $B
step bench_d45 300 python bench.py --dim 45 $B
step bench_ragged 300 python bench.py --ragged $B
step prof_modes 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --mode sum --gpus 1 --steps 5 --warmup 1 --cpu-baseline off --host-boundary off --extras off --no-extra-mode
echo done
