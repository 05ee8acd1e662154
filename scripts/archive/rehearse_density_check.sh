set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
RASR_BENCH_SAME_DEVICE=1 RASR_BENCH_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/rehearse_n2_density_check.json 2> gpurun_out/rehearse_n2.err || { tail -30 gpurun_out/rehearse_n2.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/rehearse_n2_density_check.json').read().strip().splitlines()[-1]); print(d['n_gpus'], d['value'], d.get('density_sharded'))"
