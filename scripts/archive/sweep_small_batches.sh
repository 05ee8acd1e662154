#!/bin/bash
# Chunk-size sweep at SURVEY 8(d) config 2's small batches (256 / 1024 / 4096 frames per call): the work units
# a launch is cut into (RASR_GMM_TARGET_BLOCKS) against the per-workgroup frame-operand reload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for mode in fp32 simd; do
  for f in 256 1024 4096; do
    for tb in 1024 2048 4096 8192; do
      r=$(RASR_GMM_TARGET_BLOCKS=$tb timeout -k 10 120 python scripts/ab_bench.py --mode $mode --frames $f --steps 200 --rounds 2 rasr_amd/lib/librasr_gmm.so) || exit 1
      echo "$mode frames=$f target_blocks=$tb $r"
    done
  done
done
