#!/bin/bash
# Same-card A/B of scoreSplit's per-frame-tile rotation of the chunk's mixture order (rot1) against every workgroup
# walking the chunk from its first mixture (rot0), at the headline's 32768 frames per launch; then the float parity
# tests on the rotated build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03_ab_rotate
mkdir -p $OUT
V=rasr_amd/lib/variants
timeout -k 10 500 python scripts/ab_bench.py --mode fp32 --frames 32768 --rounds 4 --steps 12 \
    $V/librasr_gmm_rot0.so $V/librasr_gmm_rot1.so > $OUT/ab_fp32.txt 2>&1 || exit $?
cat $OUT/ab_fp32.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_scores_only.py tests/test_preselection.py -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; exit $rc
