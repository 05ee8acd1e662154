#!/bin/bash
# Build kernel variants for A/B timing (scripts/ab_bench.py):
#   build_variants.sh <name> "<i8 kernel flags>" "<f32 kernel flags>" [<name> "<i8>" "<f32>"]...
# (the f32 flags also go to the split-f16 kernel TU; -D flags reach gmm_api.cc too)
# -> rasr_amd/lib/variants/librasr_gmm_<name>.so (same host objects, different kernel objects)
# VARIANT_PATCHES: patches (scripts/variants/*.patch) applied to a copy of rasr_amd/csrc the kernels are built
# from: the measured A/B code paths that are not in the product sources (scripts/variants/README.md)
set -e
cd "$(dirname "$0")/.."
make -s all
# every object except the kernel TUs and the API TU rebuilt per variant below
OTHER=$(ls build/*.o | grep -v -E "gmm_kernels_(i8|f32|split)\.o|gmm_api\.o")
mkdir -p rasr_amd/lib/variants build/variants
BASE="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off"
# the product build's per-TU flags (Makefile), so a variant differs from librasr_gmm.so only by its own flags
I8F=$(make -s print-I8FLAGS); F32F=$(make -s print-F32FLAGS); SPLITF=$(make -s print-SPLITFLAGS)
while [ $# -ge 3 ]; do
  name=$1; i8=$2; f32=$3; shift 3
  SRCDIR=rasr_amd/csrc
  if [ -n "$VARIANT_PATCHES" ]; then
    SRCDIR=build/variants/csrc_$name
    rm -rf $SRCDIR && cp -r rasr_amd/csrc $SRCDIR
    for p in $VARIANT_PATCHES; do patch -s -p1 -d $SRCDIR < $p; done
  fi
  /opt/rocm/bin/hipcc $BASE $I8F $i8 -c $SRCDIR/gmm_kernels_i8.hip -o build/variants/i8_$name.o
  /opt/rocm/bin/hipcc $BASE $F32F $f32 -c $SRCDIR/gmm_kernels_f32.hip -o build/variants/f32_$name.o
  /opt/rocm/bin/hipcc $BASE $SPLITF $f32 -c $SRCDIR/gmm_kernels_split.hip -o build/variants/split_$name.o
  defs=$(echo "$i8 $f32" | tr ' ' '\n' | grep '^-D' | tr '\n' ' ')
  /opt/rocm/bin/hipcc -O2 -std=c++17 -fPIC -ffp-contract=off -Ibuild $defs -c rasr_amd/csrc/gmm_api.cc -o build/variants/api_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o rasr_amd/lib/variants/librasr_gmm_$name.so \
      build/variants/i8_$name.o build/variants/f32_$name.o build/variants/split_$name.o build/variants/api_$name.o $OTHER -lz -pthread -ldl
  echo built $name
done
