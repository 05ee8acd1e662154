#!/bin/bash
# Round-3 closing check on HEAD: the GPU suite, smoke, and the default bench line (as the driver runs them).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN:-r03_final}
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
ALLOW_FAIL=1 step pytest 1100 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 900 python bench.py
echo done
