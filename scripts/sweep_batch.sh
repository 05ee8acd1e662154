# Frames per scorer call (RASR's buffer-size) vs throughput, fp32 and SIMD modes, one GPU:
#   bash scripts/sweep_batch.sh  -> gpurun_out/sweep_batch.txt (one bench JSON line per point)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/sweep_batch.txt
: > $out
for mode in fp32 simd; do
  for f in 256 1024 4096 8192 32768; do
    # launches per step: about 50 ms of kernel time per step at the measured rates
    per=$(python -c "print(max(1, int(50.0 / ($f * (0.00016 if '$mode' == 'fp32' else 0.00006)))))")
    echo "== $mode frames=$f launches=$per" >> $out
    timeout -k 10 240 python bench.py --mode $mode --frames $f --launches $per --steps 10 --warmup 2 \
        --cpu-baseline off --host-boundary off --no-extra-mode 2>/dev/null | tail -1 >> $out || exit 1
  done
done
python - <<'PY'
import json
for line in open("gpurun_out/sweep_batch.txt"):
    if line.startswith("{"):
        d = json.loads(line)
        r = d["roofline"]
        print(f'{d["config"]["scorer"]:24s} frames/launch {d["config"]["frames_per_launch"]:6d}: '
              f'{d["value"] / 1e6:6.2f} M frames/s, kernel {r["kernel_ms"]:.3f} ms, frac {r["frac"]:.3f}')
PY
