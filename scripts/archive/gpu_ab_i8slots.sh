# round 2: scoreI8Seg running-minimum slots (1 register per column block instead of 4) -- parity, then A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=rasr_amd/lib/variants
RASR_GMM_LIB=$PWD/$V/librasr_gmm_s1w4.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_density_sharded.py tests/test_host_protocol.py -k "simd or batch_int or batch_fast or SIMD or score_scale or single_frame or full_size or shard or protocol or node" \
    > gpurun_out/pytest_s1w4.log 2>&1 || { tail -30 gpurun_out/pytest_s1w4.log; exit 1; }
tail -1 gpurun_out/pytest_s1w4.log
timeout -k 10 700 python scripts/ab_bench.py --mode simd --rounds 3 --steps 400 --frames 32768 $V/librasr_gmm_base.so \
    $V/librasr_gmm_s1w4.so $V/librasr_gmm_s1.so $V/librasr_gmm_s4w4.so \
    > gpurun_out/ab_i8_slots.txt 2>&1 || { cat gpurun_out/ab_i8_slots.txt; exit 1; }
cat gpurun_out/ab_i8_slots.txt
