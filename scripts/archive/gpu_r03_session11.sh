#!/bin/bash
# Round-3 session 11: asynchronous prefetch in the buffered drop-in (GMM_HOST_ASYNC): the new tests, the full GPU
# suite, and the drop-in protocol throughput at RASR buffer sizes (dump and search-like consumers).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN:-r03_s11}
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
ALLOW_FAIL=1 step pytest_new 600 python -u -m pytest tests/test_host_protocol.py tests/test_host_pipeline.py -q -m gpu --timeout 120 --timeout-method thread
ALLOW_FAIL=1 step pytest 1100 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread
for t in SIMD-diagonal-maximum diagonal-maximum; do
  step dropin_$t 300 build/tests/feature_scorer_driver bench $t 4,64,512,4096 6000,65536,196608,262144 5000 160 39 0 1000
  step dropin10_$t 300 build/tests/feature_scorer_driver bench $t 64,512,4096 65536,196608,262144 5000 160 39 0 100
done
echo done
