# round 2: scoreI8Seg32 with 2 column blocks per wave (98 VGPRs, 4-5 waves per SIMD) -- parity, then A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=rasr_amd/lib/variants
RASR_GMM_LIB=$PWD/$V/librasr_gmm_cb2.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_density_sharded.py -k "simd or batch_int or batch_fast or SIMD or score_scale or single_frame or full_size or shard" \
    > gpurun_out/pytest_cb2.log 2>&1 || { tail -30 gpurun_out/pytest_cb2.log; exit 1; }
tail -2 gpurun_out/pytest_cb2.log
timeout -k 10 700 python scripts/ab_bench.py --mode simd --rounds 3 --steps 400 --frames 32768 $V/librasr_gmm_base.so \
    $V/librasr_gmm_cb2.so $V/librasr_gmm_cb2s8.so $V/librasr_gmm_cb2n4.so $V/librasr_gmm_cb4.so \
    > gpurun_out/ab_i8_cb.txt 2>&1 || { cat gpurun_out/ab_i8_cb.txt; exit 1; }
cat gpurun_out/ab_i8_cb.txt
