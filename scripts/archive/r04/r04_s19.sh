#!/bin/bash
# round-4 session 18: the generalized pipeline at two pairs in flight against the previous code
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_s19; mkdir -p $O
V="rasr_amd/lib/variants/librasr_gmm_oldpipe.so rasr_amd/lib/variants/librasr_gmm_newpipe.so"
timeout -k 10 300 python scripts/ab_bench.py --mode fp32 --frames 32768 --rounds 3 $V > $O/ab_fp32.log 2>&1 || exit 1
timeout -k 10 300 python scripts/ab_bench.py --mode fp32s --frames 32768 --rounds 3 $V > $O/ab_fp32s.log 2>&1 || exit 1
timeout -k 10 300 python scripts/ab_bench.py --mode fp32 --dim 45 --frames 32768 --rounds 3 $V > $O/ab_d45.log 2>&1 || exit 1
cat $O/ab_*.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_scores_only.py tests/test_golden.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
