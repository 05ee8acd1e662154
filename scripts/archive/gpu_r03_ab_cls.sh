#!/bin/bash
# Same-card A/B of the score-only layouts: oldcls = class tiles only (round-3 session 5 layout and kernel),
# newcls = class + mixed tiles, mix100 = the new kernel on class tiles only (planner mixed cost 100); simd = the
# key-layout kernel (SIMD with best densities) of old and new builds, for regressions.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r03_ab_cls2
mkdir -p $OUT
V=rasr_amd/lib/variants
for mode in bint simds simd; do
  timeout -k 10 500 python scripts/ab_bench.py --mode $mode --rounds 3 --steps 20 \
      $V/librasr_gmm_oldcls.so $V/librasr_gmm_newcls.so $V/librasr_gmm_mix100.so > $OUT/ab_$mode.txt 2>&1 || exit $?
  cat $OUT/ab_$mode.txt
done
