# round 2: D = 45 (config 3) on the 16-row (16x16x32, K 160) vs the 32-row (32x32x16, K 144) split kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=rasr_amd/lib/librasr_gmm.so
timeout -k 10 900 python scripts/ab_bench.py --mode fp32 --dim 45 --rounds 3 --steps 200 --frames 32768 $L:split32 $L:split16 \
    > gpurun_out/ab_d45_shape.txt 2>&1 || { cat gpurun_out/ab_d45_shape.txt; exit 1; }
cat gpurun_out/ab_d45_shape.txt
