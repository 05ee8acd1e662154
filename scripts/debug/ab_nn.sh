#!/bin/bash
# A/B of NN GEMM variant libraries: parity (tests/test_nn_scorer.py) then bench --mode nn, per variant
set -e
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for v in "$@"; do
  RASR_GMM_LIB=$PWD/rasr_amd/lib/variants/librasr_gmm_$v.so timeout -k 10 200 python -u -m pytest tests/test_nn_scorer.py -x -q --timeout 150 --timeout-method thread -m gpu > gpurun_out/ab_nn_test_$v.log 2>&1
  RASR_GMM_LIB=$PWD/rasr_amd/lib/variants/librasr_gmm_$v.so timeout -k 10 200 python -u bench.py --mode nn --cpu-baseline off --steps 10 > gpurun_out/ab_nn_$v.log 2>&1
  echo "$v $(tail -n 1 gpurun_out/ab_nn_test_$v.log) $(tail -n 1 gpurun_out/ab_nn_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), round(d["roofline"]["kernel_ms"],4), round(d["roofline"]["frac"],4))')"
done
