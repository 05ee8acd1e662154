#!/bin/bash
# round-4 session 15: parallel frame preparation (tests, hashes against the previous build, small-call latency)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_s15; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
V="rasr_amd/lib/variants/librasr_gmm_prep2.so rasr_amd/lib/variants/librasr_gmm_tb8192.so"
for m in fp32 simd sum; do timeout -k 10 300 python scripts/ab_bench.py --mode $m --frames 32768 --rounds 2 $V > $O/ab_$m.log 2>&1 || exit 1; done
timeout -k 10 300 python scripts/ab_bench.py --mode simd --frames 256 --rounds 2 $V > $O/ab_simd256.log 2>&1 || exit 1
cat $O/ab_*.log
timeout -k 10 300 python scripts/host_latency.py > $O/host_latency.log 2>&1 || exit 1
cat $O/host_latency.log
timeout -k 10 120 build/tests/feature_scorer_driver bench diagonal-maximum 1,4,64 1500,6000,65536 5000 160 39 0 1000 > $O/dropin.log 2>&1 || exit 1
timeout -k 10 120 build/tests/feature_scorer_driver bench SIMD-diagonal-maximum 1,4,64 1500,6000,65536 5000 160 39 0 1000 > $O/dropin_simd.log 2>&1 || exit 1
cat $O/dropin.log $O/dropin_simd.log
