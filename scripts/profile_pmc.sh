#!/bin/bash
# PMC passes (one rocprofv3 --pmc run per counter group, no tracing domains) on a short bench run.
# usage: scripts/profile_pmc.sh <mode> [frames]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
MODE=${1:-fp32}; FRAMES=${2:-0}
OUT=gpurun_out/pmc_$MODE
mkdir -p $OUT
export TMPDIR=/tmp
PASSES=(
  "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
  "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD"
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY"
  "SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCC_HIT_sum TCC_MISS_sum"
)
# PMC_EXTRA: one more pass (e.g. "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS")
[ -n "$PMC_EXTRA" ] && PASSES+=("$PMC_EXTRA")
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  echo "=== pass $i: $p"
  timeout -k 10 300 rocprofv3 --pmc $p -d $OUT/p$i -o run --output-format csv -- \
      python bench.py --mode $MODE --steps 2 --warmup 1 --launches 2 --cpu-baseline off --host-boundary off --extras off --no-extra-mode ${FRAMES:+--frames $FRAMES} > $OUT/p$i.log 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $OUT/p$i.log; exit $rc; fi
done
echo done
