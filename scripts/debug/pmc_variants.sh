#!/bin/bash
# SQ/TCC counter passes per library variant (GPU box only): pmc_variants.sh v1 v2 ...
# -> gpurun_out/pmcv_<v>/p<i>/..., summarised by scripts/pmc_summary.py
set -u
V=rasr_amd/lib/variants
export TMPDIR=/tmp
PASSES=(
  "GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"
  "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_LDS SQ_WAIT_INST_LDS"
  "TCC_HIT_sum TCC_MISS_sum"
)
for v in "$@"; do
  i=0
  for p in "${PASSES[@]}"; do
    i=$((i+1))
    OUT=gpurun_out/pmcv_$v
    mkdir -p $OUT
    RASR_GMM_LIB=$V/librasr_gmm_$v.so timeout -k 10 120 rocprofv3 --pmc $p -d $OUT/p$i -o run --output-format csv -- \
      python bench.py --mode fp32 --steps 3 --warmup 1 --cpu-baseline off --no-extra-mode > $OUT/p$i.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$v pass $i rc=$rc"; tail -5 $OUT/p$i.log; exit $rc; fi
  done
  python scripts/pmc_summary.py $OUT scoreSplit > $OUT/summary.json && echo "== $v" && python - $OUT/summary.json <<'PY'
import json,sys
d=json.load(open(sys.argv[1])); c=d["counters"]
wc=c.get("SQ_WAVE_CYCLES",1)
print(f"  dur {d['avg_duration_s']*1e3:.3f} ms clk {d.get('effective_clock_ghz',0):.2f} GHz mfma_busy {d.get('mfma_busy_frac',0):.3f} "
      f"wait_any {c.get('SQ_WAIT_ANY',0)/wc:.3f} wait_inst {c.get('SQ_WAIT_INST_ANY',0)/wc:.3f} active {c.get('SQ_ACTIVE_INST_ANY',0)/wc:.3f} "
      f"valu/mfma {c.get('SQ_INSTS_VALU',0)/max(1,c.get('SQ_INSTS_MFMA',1)):.2f} l2hit {d.get('l2_hit_rate',0):.3f} "
      f"l2req {c.get('TCC_HIT_sum',0)+c.get('TCC_MISS_sum',0):.3e} waves {c.get('SQ_WAVES',0):.0f}")
PY
done
