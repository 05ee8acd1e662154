# round 2: NN tanh epilogue (fast vs libm tanhf) -- parity of the product build, then bench --mode nn --nn-activation tanh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_nn_scorer.py -x -q --timeout 150 --timeout-method thread -m gpu > gpurun_out/nn_tanh_tests.log 2>&1 || { tail -20 gpurun_out/nn_tanh_tests.log; exit 1; }
tail -1 gpurun_out/nn_tanh_tests.log
for v in ft noft ft noft; do
  RASR_GMM_LIB=$PWD/rasr_amd/lib/variants/librasr_gmm_$v.so timeout -k 10 200 python -u bench.py --mode nn --nn-activation tanh --cpu-baseline off --steps 10 > gpurun_out/ab_nn_tanh_$v.log 2>&1 || exit 1
  echo "$v $(tail -n 1 gpurun_out/ab_nn_tanh_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), round(d["roofline"]["kernel_ms"],4), round(d["roofline"]["frac"],4))')"
done
