# round 2: NN input conversion kernel (one workgroup per frame, bf16 pairs) -- parity, then wall-clock A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=rasr_amd/lib/variants
RASR_GMM_LIB=$PWD/$V/librasr_gmm_newprep.so timeout -k 10 300 python -u -m pytest tests/test_nn_scorer.py -x -q --timeout 150 --timeout-method thread -m gpu > gpurun_out/nn_prep_tests.log 2>&1 || { tail -20 gpurun_out/nn_prep_tests.log; exit 1; }
tail -1 gpurun_out/nn_prep_tests.log
for v in newprep oldprep newprep oldprep; do
  RASR_GMM_LIB=$PWD/$V/librasr_gmm_$v.so timeout -k 10 200 python -u bench.py --mode nn --cpu-baseline off --steps 20 > gpurun_out/ab_nn_prep_$v.log 2>&1 || exit 1
  echo "$v $(tail -n 1 gpurun_out/ab_nn_prep_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), round(d["ms_per_step"],3), round(d["roofline"]["kernel_ms"],4))')"
done
