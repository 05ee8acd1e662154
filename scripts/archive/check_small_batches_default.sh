cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_chunks.log 2>&1 || { tail -20 gpurun_out/pytest_chunks.log; exit 1; }
tail -2 gpurun_out/pytest_chunks.log
for mode in fp32 simd; do for f in 256 1024 4096; do
  r=$(timeout -k 10 120 python scripts/ab_bench.py --mode $mode --frames $f --steps 200 --rounds 2 rasr_amd/lib/librasr_gmm.so) || exit 1
  echo "$mode frames=$f default $r"
done; done
