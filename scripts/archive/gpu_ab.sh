# A/B kernel timing of the default library against variants built by scripts/build_variants.sh:
#   gpu_ab.sh <mode> <variant>...   -> gpurun_out/ab_<mode>.txt
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
mode=$1; shift
libs="rasr_amd/lib/librasr_gmm.so"
for v in "$@"; do
  case $v in :*) libs="$libs rasr_amd/lib/librasr_gmm.so$v" ;; *) libs="$libs rasr_amd/lib/variants/librasr_gmm_$v.so" ;; esac
done
timeout -k 10 500 python scripts/ab_bench.py --mode $mode --rounds 3 --steps 40 --frames 32768 $libs \
    > gpurun_out/ab_$mode.txt 2>&1 || { tail -20 gpurun_out/ab_$mode.txt; exit 1; }
cat gpurun_out/ab_$mode.txt
