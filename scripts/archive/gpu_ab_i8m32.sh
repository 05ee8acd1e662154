# round 2: 32x32x32 quantized kernel (scoreI8Seg32) -- parity of the variant, then A/B against the product kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=rasr_amd/lib/variants
RASR_GMM_LIB=$PWD/$V/librasr_gmm_m32.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "simd or batch_int or batch_fast or SIMD or score_scale or single_frame or full_size" \
    > gpurun_out/pytest_m32.log 2>&1 || { tail -30 gpurun_out/pytest_m32.log; exit 1; }
tail -3 gpurun_out/pytest_m32.log
timeout -k 10 600 python scripts/ab_bench.py --mode simd --rounds 3 --steps 40 --frames 32768 rasr_amd/lib/librasr_gmm.so \
    $V/librasr_gmm_m32.so $V/librasr_gmm_m32n4.so $V/librasr_gmm_m32i6.so $V/librasr_gmm_m32w4.so \
    > gpurun_out/ab_i8_m32.txt 2>&1 || { cat gpurun_out/ab_i8_m32.txt; exit 1; }
cat gpurun_out/ab_i8_m32.txt
