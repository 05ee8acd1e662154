#!/bin/bash
# round-4 session 23: one-wave 64-frame workgroups for quantized calls of <= 64 frames
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_s23; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python scripts/host_latency.py --types SIMD-diagonal-maximum,batch-diagonal-maximum-int > $O/host_latency.log 2>&1 || exit 1
RASR_GMM_TARGET_BLOCKS=8192 timeout -k 10 200 python scripts/host_latency.py --types SIMD-diagonal-maximum --sizes 1,4,16,64 > $O/host_latency_tb8192.log 2>&1 || exit 1
cat $O/host_latency.log $O/host_latency_tb8192.log
timeout -k 10 120 build/tests/feature_scorer_driver bench SIMD-diagonal-maximum 1,4,64 1500,6000,65536 5000 160 39 0 1000 > $O/dropin_simd.log 2>&1 || exit 1
cat $O/dropin_simd.log
