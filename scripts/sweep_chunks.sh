#!/bin/bash
# Sweep of the chunk-count target (RASR_GMM_TARGET_BLOCKS) and frames per step for the headline
# fp32 bench line; one bench.py process per point, each under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for f in ${FRAMES:-32768 65536}; do
  for tb in ${BLOCKS:-4096 8192 16384 32768}; do
    RASR_GMM_TARGET_BLOCKS=$tb timeout -k 10 180 python bench.py --frames $f --steps 20 --warmup 3 --no-extra-mode \
      --cpu-baseline off > gpurun_out/sweep_${f}_${tb}.json 2> gpurun_out/sweep_${f}_${tb}.err || exit $?
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['value']/1e6,3), 'M frames/s', round(d['roofline']['frac'],4), round(d['roofline']['kernel_ms'],3), 'ms')" \
      gpurun_out/sweep_${f}_${tb}.json $f $tb | tee -a gpurun_out/sweep.txt
  done
done
