#!/bin/bash
# Same-card A/B of the score-only mixed step's lag (columns blocks between a block's MFMAs and its epilogue):
# newcls = lag 1, lag2, lag3; oldcls = class tiles only (the round-3 session-5 kernel).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03_ab_lag
mkdir -p $OUT
V=rasr_amd/lib/variants
for mode in bint simds; do
  timeout -k 10 500 python scripts/ab_bench.py --mode $mode --rounds 3 --steps 20 \
      $V/librasr_gmm_oldcls.so $V/librasr_gmm_newcls.so $V/librasr_gmm_lag2.so $V/librasr_gmm_lag3.so > $OUT/ab_$mode.txt 2>&1 || exit $?
  cat $OUT/ab_$mode.txt
done
