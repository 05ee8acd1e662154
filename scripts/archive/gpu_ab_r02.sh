# A/B timing of library variants built by scripts/build_variants.sh (round 2 experiments)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=rasr_amd/lib/variants
timeout -k 10 400 python scripts/ab_bench.py --mode simd --rounds 3 --steps 40 --frames 32768 rasr_amd/lib/librasr_gmm.so \
    $V/librasr_gmm_d2.so $V/librasr_gmm_d4.so $V/librasr_gmm_d8.so $V/librasr_gmm_d14.so $V/librasr_gmm_nil.so \
    > gpurun_out/ab_simd_diag.txt 2>&1 || exit $?
cat gpurun_out/ab_simd_diag.txt
