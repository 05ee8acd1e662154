#!/bin/bash
# correctness (ragged multi-tile case) + timing of the split-kernel variants; GPU box only
set -u
V=rasr_amd/lib/variants
mkdir -p gpurun_out
for v in "$@"; do
  echo "== $v"
  QUICK=1 RASR_GMM_LIB=$V/librasr_gmm_$v.so timeout -k 10 100 python scripts/debug/split_diag.py > gpurun_out/diag_$v.log 2>&1
  rc=$?
  grep -v amdgpu.ids gpurun_out/diag_$v.log | head -6
  [ $rc -eq 0 ] || exit $rc
done
libs=""
for v in "$@"; do libs="$libs $V/librasr_gmm_$v.so"; done
timeout -k 10 300 python scripts/ab_bench.py --mode fp32 --rounds 2 $libs
