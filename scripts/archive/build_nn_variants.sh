#!/bin/bash
# NN GEMM variants for A/B timing: build_nn_variants.sh <name> "<nn_kernels.hip flags>" [...]
# -> rasr_amd/lib/variants/librasr_gmm_<name>.so (select with RASR_GMM_LIB; every other object as built)
set -e
cd "$(dirname "$0")/.."
make -s all
mkdir -p rasr_amd/lib/variants build/variants
OBJS=$(ls build/*.o | grep -v nn_kernels.o)
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $flags \
      -c rasr_amd/csrc/nn_kernels.hip -o build/variants/nn_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o rasr_amd/lib/variants/librasr_gmm_$name.so \
      $OBJS build/variants/nn_$name.o -lz
  echo built $name
done
