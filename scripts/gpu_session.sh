#!/bin/bash
# One GPU session on the gpurun box: each step under its own time limit, stop at the first failure.
#   RUN=<name> STEPS="pytest smoke bench prof" scripts/gpu_session.sh
# Outputs under gpurun_out/$RUN/ (copy what is to be kept into profiles/).
#   pytest  : the -m gpu suite (PYTEST_ARGS overrides the selection, e.g. "tests/test_rccl_exchange.py")
#   smoke   : __graft_entry__.smoke()
#   bench   : python bench.py (BENCH_ARGS appended)
#   prof    : rocprofv3 --kernel-trace --stats over bench.py (BENCH_ARGS appended)
#   ab-MODE : scripts/ab_bench.py --mode MODE over AB_LIBS (default: the variant libraries), AB_ARGS appended
#   pmc-MODE: scripts/profile_pmc.sh MODE (one rocprofv3 --pmc pass per counter group, gpurun_out/pmc_MODE)
#   line-X  : one other bench line, timed alone (X: sum sums d45 d45s pint pfloat nn ragged covm covn covms covsum)
#   rehearse: the N > 1 bench flow on this one GPU (2 ranks on device 0, gloo in place of RCCL): headline, the
#             fenced density-sharded / C-ABI children, the line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN:-session}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -5 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in ${STEPS:-pytest smoke}; do
  case $s in
    pytest) step pytest 1100 python -u -m pytest ${PYTEST_ARGS:-tests -m gpu} -q --timeout 120 --timeout-method thread -p no:cacheprovider ;;
    smoke)  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  step bench 900 python bench.py ${BENCH_ARGS} ;;
    prof)   step prof 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python bench.py ${BENCH_ARGS} ;;
    ab-*)   step "$s" 900 python scripts/ab_bench.py --mode "${s#ab-}" ${AB_ARGS} ${AB_LIBS:-rasr_amd/lib/variants/*.so} ;;
    pmc-*)  step "$s" 1000 bash scripts/profile_pmc.sh "${s#pmc-}" ;;
    rehearse) RASR_BENCH_SAME_DEVICE=1 RASR_BENCH_BACKEND=gloo step rehearse 420 python bench.py --gpus 2 --steps 3 \
                --warmup 1 --no-extra-mode --host-boundary off ;;
    line-*)
      B="--gpus 1 --steps 20 --warmup 3 --cpu-baseline off --host-boundary off --extras off --no-extra-mode"
      case ${s#line-} in
        sum) A="--mode sum" ;; sums) A="--mode sum --no-best" ;; d45) A="--dim 45" ;;
        d45s) A="--dim 45 --mode simd-scores" ;; pint) A="--mode presel-int" ;; pfloat) A="--mode presel-float" ;;
        nn) A="--mode nn" ;; ragged) A="--ragged" ;;
        covm) A="--tying mixture-specific" ;; covn) A="--tying none" ;; covms) A="--tying mixture-specific --mode simd" ;;
        covsum) A="--tying none --mode sum" ;;
        *) echo "unknown line $s"; exit 2 ;;
      esac
      step "$s" 300 python bench.py $A $B ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo done
