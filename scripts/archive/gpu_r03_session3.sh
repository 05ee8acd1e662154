#!/bin/bash
# Round-3 GPU session 3: parity tests and smoke on the pipelined scoreI8Seg build, PMC summaries for this build's
# kernels (the kernel id changed), the default bench line and its rocprofv3 kernel-trace summary.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN:-r03_s3}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>; ALLOW_FAIL=1: a plain failure (rc 1: failed tests) does not stop the run
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
step pmc_fp32 600 bash scripts/profile_pmc.sh fp32
step pmc_simd 600 bash scripts/profile_pmc.sh simd
step pmc_presel 600 bash scripts/profile_pmc.sh presel-int
python scripts/pmc_summary.py gpurun_out/pmc_fp32 scoreSplit --json $OUT/pmc_fp32.json > /dev/null || exit 1
python scripts/pmc_summary.py gpurun_out/pmc_simd scoreI8 --json $OUT/pmc_simd.json > /dev/null || exit 1
python scripts/pmc_summary.py gpurun_out/pmc_presel-int scoreI8 --json $OUT/pmc_presel_int.json > /dev/null || exit 1
cp $OUT/pmc_fp32.json $OUT/pmc_simd.json profiles/
step bench 900 python bench.py --gpus 1 --steps 20 --warmup 5
step prof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off --host-boundary off --extras off
echo done
