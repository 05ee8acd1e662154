# round 2: preselection-batch-int with compressed mask tables (occupancy 2 -> 5 workgroups per CU) -- parity, A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=rasr_amd/lib/variants
RASR_GMM_LIB=$PWD/$V/librasr_gmm_nib.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_preselection.py > gpurun_out/pytest_nib.log 2>&1 || { tail -30 gpurun_out/pytest_nib.log; exit 1; }
tail -1 gpurun_out/pytest_nib.log
for v in nib base nib base; do
  RASR_GMM_LIB=$PWD/$V/librasr_gmm_$v.so timeout -k 10 300 python -u bench.py --mode presel-int --steps 10 --warmup 2 --cpu-baseline off --host-boundary off --no-extra-mode > gpurun_out/ab_presel_$v.log 2>&1 || exit 1
  echo "$v $(tail -n 1 gpurun_out/ab_presel_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]/1e6,3), round(d["roofline"]["kernel_ms"],4))')"
done
