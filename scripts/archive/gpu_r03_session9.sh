#!/bin/bash
# Round-3 session 9: class + mixed tiles in the score-only layout (SIMD scores-only, batch-int): parity tests,
# then the score-only bench lines and the kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN:-r03_s9}
mkdir -p $OUT
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 $OUT/$name.log
  if [ $rc -eq 1 ] && [ -n "$ALLOW_FAIL" ]; then return 0; fi
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest_so 400 python -u -m pytest tests/test_scores_only.py tests/test_batch_int_score_only.py -x -q -m gpu --timeout 120 --timeout-method thread
for mode in simd-scores bint; do
  step bench_$mode 300 python bench.py --mode $mode --steps 20 --warmup 5 --cpu-baseline off --extras off --host-boundary off --no-extra-mode
done
ALLOW_FAIL=1 step pytest 1100 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread
echo done
