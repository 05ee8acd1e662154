#!/bin/bash
# hybrid-DNN split-K A/B (nnGemm128 hidden layers): all-layer time per call size, by RASR_NN_MAX_SPLIT and
# against no split (RASR_NN_SPLIT_K=0) and the small-call kernel (RASR_NN_SMALL_FRAMES)
timeout -k 10 400 python -u -m pytest tests/test_nn_scorer.py tests/test_nn_integration.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/nn_tests.log 2>&1; rc=$?; tail -3 gpurun_out/nn_tests.log; [ $rc = 0 ] || exit $rc
run() {  # label frames env...
  local l=$1 f=$2; shift 2
  env "$@" timeout -k 10 120 python bench.py --mode nn --frames $f --launches 16 --steps 10 --warmup 2 --no-extra-mode --cpu-baseline off --host-boundary off --extras off > gpurun_out/ab_${l}_$f.json || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_${l}_$f.json'));r=d['roofline'];print('$l', $f, round(d['value']/1e6,2), 'M/s', round(r['kernel_ms'],4))"
}
for f in 96 128 160 193 256 384 512 768 1024; do
  run split4 $f RASR_NN_SMALL_FRAMES=64 RASR_NN_MAX_SPLIT=4
  run split8 $f RASR_NN_SMALL_FRAMES=64 RASR_NN_MAX_SPLIT=8
done
for f in 96 128 160; do
  run small $f RASR_NN_SMALL_FRAMES=1000
done
