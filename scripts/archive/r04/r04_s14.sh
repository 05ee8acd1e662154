#!/bin/bash
# round-4 session 14: split chunk cap on the other split lines, drop-in with the page-locked 1-frame slot,
# HIP API timeline of a 1-frame host call
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_s14; mkdir -p $O
V="rasr_amd/lib/variants/librasr_gmm_tb2048.so rasr_amd/lib/variants/librasr_gmm_tb8192.so"
timeout -k 10 300 python scripts/ab_bench.py --mode sum --frames 32768 --rounds 3 $V > $O/ab_sum.log 2>&1 || exit 1
timeout -k 10 300 python scripts/ab_bench.py --mode fp32 --dim 45 --frames 32768 --rounds 3 $V > $O/ab_d45.log 2>&1 || exit 1
timeout -k 10 300 python scripts/ab_bench.py --mode fp32s --frames 32768 --rounds 3 $V > $O/ab_fp32s.log 2>&1 || exit 1
timeout -k 10 300 python scripts/ab_bench.py --mode fp32 --frames 1024 --rounds 3 $V > $O/ab_1024.log 2>&1 || exit 1
cat $O/ab_*.log
timeout -k 10 120 build/tests/feature_scorer_driver bench diagonal-maximum 1,4,64 1500,6000,65536 5000 160 39 0 1000 > $O/dropin.log 2>&1 || exit 1
timeout -k 10 120 build/tests/feature_scorer_driver bench SIMD-diagonal-maximum 1,4,64 1500,6000,65536 5000 160 39 0 1000 > $O/dropin_simd.log 2>&1 || exit 1
cat $O/dropin.log $O/dropin_simd.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --hip-runtime-trace --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/$O/api -o run -- python3 $GRAFT_REPO_ROOT/scripts/host_latency.py --types diagonal-maximum --sizes 1,4 --calls 200 > $GRAFT_REPO_ROOT/$O/api.log 2>&1 || exit 1
ls -R $GRAFT_REPO_ROOT/$O/api | head -20
