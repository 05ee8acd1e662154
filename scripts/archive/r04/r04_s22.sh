#!/bin/bash
# round-4 session 18: 512-frame workgroups (4 waves x 128 frames) against 256
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_s22; mkdir -p $O
V="rasr_amd/lib/variants/librasr_gmm_fpb256.so rasr_amd/lib/variants/librasr_gmm_fpb512.so"
timeout -k 10 300 python scripts/ab_bench.py --mode fp32 --frames 32768 --rounds 3 $V > $O/ab_fp32.log 2>&1 || exit 1
timeout -k 10 300 python scripts/ab_bench.py --mode fp32s --frames 32768 --rounds 3 $V > $O/ab_fp32s.log 2>&1 || exit 1
timeout -k 10 300 python scripts/ab_bench.py --mode fp32 --dim 45 --frames 32768 --rounds 3 $V > $O/ab_d45.log 2>&1 || exit 1
cat $O/ab_*.log
RASR_GMM_LIB=$PWD/rasr_amd/lib/variants/librasr_gmm_fpb512.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
