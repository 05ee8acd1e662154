#!/bin/bash
# Round-2 closing GPU session after the NN epilogue work (GMM kernels unchanged since run6, whose PMC summaries
# are this build's): parity tests, smoke, the default bench line, the rocprofv3 kernel-trace summary of the same
# command, the NN bench line and its kernel summary.
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
  tail -2 $OUT/$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step pytest 1200 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --gpus 1 --steps 20 --warmup 5
step prof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off --host-boundary off
step bench_nn 600 python bench.py --mode nn --steps 20 --warmup 3
step prof_nn 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_nn -o run --output-format csv -- python bench.py --mode nn --steps 20 --warmup 3
echo done
