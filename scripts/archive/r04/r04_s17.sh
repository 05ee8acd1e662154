#!/bin/bash
# round-4 session 17: the emit's share (diagnostic variant), emit-flat, 256-frame tiles for small quantized calls
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_s17; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python scripts/ab_bench.py --mode fp32 --frames 32768 --rounds 3 rasr_amd/lib/variants/*.so > $O/ab_fp32.log 2>&1 || exit 1
cat $O/ab_fp32.log
timeout -k 10 300 python scripts/ab_bench.py --mode simd --frames 256 --rounds 3 rasr_amd/lib/librasr_gmm.so rasr_amd/lib/variants/librasr_gmm_prod.so > $O/ab_simd256.log 2>&1 || exit 1
timeout -k 10 300 python scripts/ab_bench.py --mode bint --frames 64 --rounds 3 rasr_amd/lib/librasr_gmm.so rasr_amd/lib/variants/librasr_gmm_prod.so > $O/ab_bint64.log 2>&1 || exit 1
cat $O/ab_simd256.log $O/ab_bint64.log
timeout -k 10 300 python scripts/host_latency.py --types SIMD-diagonal-maximum > $O/host_latency.log 2>&1 || exit 1
cat $O/host_latency.log
