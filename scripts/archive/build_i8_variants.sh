#!/bin/bash
# Quantized-kernel variants for A/B timing: build_i8_variants.sh <name> "<gmm_kernels_i8.hip flags>" [...]
# -> rasr_amd/lib/variants/librasr_gmm_<name>.so (select with RASR_GMM_LIB; every other object as built)
set -e
cd "$(dirname "$0")/.."
make -s all
mkdir -p rasr_amd/lib/variants build/variants
OBJS=$(ls build/*.o | grep -v gmm_kernels_i8.o)
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -mllvm -amdgpu-mfma-vgpr-form $flags \
      -c rasr_amd/csrc/gmm_kernels_i8.hip -o build/variants/i8_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o rasr_amd/lib/variants/librasr_gmm_$name.so \
      $OBJS build/variants/i8_$name.o -lz -pthread -lrccl
  echo built $name
done
