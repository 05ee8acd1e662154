# round 2: scoreSplit running-minimum slots -- parity of the 1-slot variant, then A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=rasr_amd/lib/variants
RASR_GMM_LIB=$PWD/$V/librasr_gmm_ssl1.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_density_sharded.py -k "fp32 or float or split or full_size or shard or scales or edge" \
    > gpurun_out/pytest_ssl1.log 2>&1 || { tail -30 gpurun_out/pytest_ssl1.log; exit 1; }
tail -1 gpurun_out/pytest_ssl1.log
timeout -k 10 900 python scripts/ab_bench.py --mode fp32 --rounds 3 --steps 200 --frames 32768 $V/librasr_gmm_base.so \
    $V/librasr_gmm_ssl1.so $V/librasr_gmm_ssl2.so > gpurun_out/ab_split_slots.txt 2>&1 || { cat gpurun_out/ab_split_slots.txt; exit 1; }
cat gpurun_out/ab_split_slots.txt
