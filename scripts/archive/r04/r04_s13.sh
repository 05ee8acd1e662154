#!/bin/bash
# round-4 session 13: chunk-cap / emit A/B, the small host-call path (tests, latency on/off, drop-in on/off)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_s13; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python scripts/host_latency.py > $O/host_latency.log 2>&1 || exit 1
RASR_GMM_SMALL_HOST=0 timeout -k 10 300 python scripts/host_latency.py > $O/host_latency_off.log 2>&1 || exit 1
cat $O/host_latency.log $O/host_latency_off.log
timeout -k 10 120 build/tests/feature_scorer_driver bench diagonal-maximum 1,4,64 1500,6000,65536 5000 160 39 0 1000 > $O/dropin.log 2>&1 || exit 1
RASR_GMM_SMALL_HOST=0 timeout -k 10 120 build/tests/feature_scorer_driver bench diagonal-maximum 1,4,64 1500,6000,65536 5000 160 39 0 1000 > $O/dropin_off.log 2>&1 || exit 1
cat $O/dropin.log $O/dropin_off.log
timeout -k 10 400 python scripts/ab_bench.py --mode fp32 --frames 32768 --rounds 3 rasr_amd/lib/variants/*.so > $O/ab_fp32.log 2>&1 || exit 1
timeout -k 10 300 python scripts/ab_bench.py --mode fp32 --frames 8192 --rounds 3 rasr_amd/lib/variants/librasr_gmm_tb*.so > $O/ab_fp32_8192.log 2>&1 || exit 1
cat $O/ab_fp32.log $O/ab_fp32_8192.log
