# round 2: diagonal-sum interleave ratios (VALU per MFMA in the two halves of a tile step)
# (the GMM_SUM_IL1 / GMM_SUM_IL2 switches the variants were built with were removed again after this A/B: no gain)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=rasr_amd/lib/variants
timeout -k 10 900 python scripts/ab_bench.py --mode sum --rounds 3 --steps 120 --frames 32768 $V/librasr_gmm_sbase.so \
    $V/librasr_gmm_s46.so $V/librasr_gmm_s68.so $V/librasr_gmm_s58.so > gpurun_out/ab_sum_il.txt 2>&1 || { cat gpurun_out/ab_sum_il.txt; exit 1; }
cat gpurun_out/ab_sum_il.txt
