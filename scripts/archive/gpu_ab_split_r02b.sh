# round 2: scoreSplit MFMA-order / priority A/B (library variants from scripts/build_variants.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=rasr_amd/lib/variants
timeout -k 10 900 python scripts/ab_bench.py --mode fp32 --rounds 3 --steps 200 --frames 32768 \
    $V/librasr_gmm_base.so $V/librasr_gmm_prio.so $V/librasr_gmm_ord1.so $V/librasr_gmm_prord.so \
    > gpurun_out/ab_split_order_prio.txt 2>&1 || { cat gpurun_out/ab_split_order_prio.txt; exit 1; }
cat gpurun_out/ab_split_order_prio.txt
