#!/bin/bash
# round-4 session 21: preselection-batch-float at 128 frames per wave
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_s21; mkdir -p $O
V="rasr_amd/lib/variants/librasr_gmm_pnf4.so rasr_amd/lib/variants/librasr_gmm_pnf8.so"
timeout -k 10 300 python scripts/ab_bench.py --mode pfloat --frames 32768 --rounds 3 $V > $O/ab_pfloat.log 2>&1 || exit 1
timeout -k 10 300 python scripts/ab_bench.py --mode pfloat --frames 32768 --dim 45 --rounds 2 $V > $O/ab_pfloat45.log 2>&1 || exit 1
cat $O/ab_*.log
RASR_GMM_LIB=$PWD/rasr_amd/lib/variants/librasr_gmm_pnf8.so timeout -k 10 600 python -u -m pytest tests/test_preselection.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_pnf8.log 2>&1 || { tail -30 $O/pytest_pnf8.log; exit 1; }
tail -2 $O/pytest_pnf8.log
