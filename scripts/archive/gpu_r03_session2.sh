#!/bin/bash
# Round-3 GPU session 2: parity tests on the housekeeping build, PMC summaries for the production kernels (and the
# masked preselection-batch-int kernel), the scoreSplit chunk-size A/B (HBM fetch / clock / time per arm), the
# default bench line and its rocprofv3 kernel-trace summary.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN:-r03_s2}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 $OUT/$name.log
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
step pmc_fp32 600 bash scripts/profile_pmc.sh fp32
step pmc_simd 600 bash scripts/profile_pmc.sh simd
step pmc_presel 600 bash scripts/profile_pmc.sh presel-int
python scripts/pmc_summary.py gpurun_out/pmc_fp32 scoreSplit --json $OUT/pmc_fp32.json > /dev/null || exit 1
python scripts/pmc_summary.py gpurun_out/pmc_simd scoreI8 --json $OUT/pmc_simd.json > /dev/null || exit 1
python scripts/pmc_summary.py gpurun_out/pmc_presel-int scoreI8 --json $OUT/pmc_presel_int.json > /dev/null || exit 1
cp $OUT/pmc_fp32.json $OUT/pmc_simd.json profiles/
# scoreSplit chunk size (mixtures per XCD work unit): the model re-fetch beyond L2 vs clock and time
for tb in 4096 8192 16384 32768; do
  export RASR_GMM_TARGET_BLOCKS=$tb
  step ab_tb${tb}_fetch 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/ab_tb${tb}_fetch -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --launches 2 --cpu-baseline off --host-boundary off --extras off --no-extra-mode
  step ab_tb${tb}_clock 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum -d $OUT/ab_tb${tb}_clock -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --launches 2 --cpu-baseline off --host-boundary off --extras off --no-extra-mode
  step ab_tb${tb}_time 300 python bench.py --steps 20 --warmup 5 --cpu-baseline off --host-boundary off --extras off --no-extra-mode
done
unset RASR_GMM_TARGET_BLOCKS
step bench 900 python bench.py --gpus 1 --steps 20 --warmup 5
step prof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off --host-boundary off --extras off
echo done
