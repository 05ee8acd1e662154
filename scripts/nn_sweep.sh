#!/bin/bash
# hybrid-DNN all-layer time per call size (bench.py --mode nn --frames F), with the kernel choice forced
# by RASR_NN_TILE128_WGS (0: nnGemm8p for every layer beyond the small-call range; 100000: nnGemm128)
set -e
out=gpurun_out/nnsweep; mkdir -p $out
for w in ${WS:-default 0 100000}; do
  for f in 257 512 1024 2048 3072 4096 6144 8192 32768; do
    if [ $w = default ]; then env=""; else env="RASR_NN_TILE128_WGS=$w"; fi
    env $env timeout -k 10 120 python bench.py --mode nn --frames $f --launches 16 --steps 10 --warmup 2 --no-extra-mode --cpu-baseline off --host-boundary off --extras off > $out/w${w}_f$f.json
    python -c "import json;d=json.load(open('$out/w${w}_f$f.json'));r=d['roofline'];print('$w', $f, round(d['value']/1e6,2), 'M/s', round(r['kernel_ms'],4), round(r['frac'],3))"
  done
done
# the small-call boundary: nnGemmSmall (default, <= NN_SMALL_FRAMES) against the tile kernels (RASR_NN_SMALL_FRAMES=0)
if [ -n "$SMALL" ]; then
  for s in default 0; do
    for f in 64 128 192 256; do
      if [ $s = default ]; then env=""; else env="RASR_NN_SMALL_FRAMES=$s"; fi
      env $env timeout -k 10 120 python bench.py --mode nn --frames $f --launches 16 --steps 10 --warmup 2 --no-extra-mode --cpu-baseline off --host-boundary off --extras off > $out/s${s}_f$f.json
      python -c "import json;d=json.load(open('$out/s${s}_f$f.json'));r=d['roofline'];print('small=$s', $f, round(d['value']/1e6,2), 'M/s', round(r['kernel_ms'],4), round(r['frac'],3))"
    done
  done
fi
