#!/bin/bash
# timing only (no correctness check) of library variants: ab_only.sh <mode> v1 v2[:split16] ...
V=rasr_amd/lib/variants
mode=$1; shift
libs=""
for v in "$@"; do
  name=${v%%:*}; opt=""
  [ "$name" != "$v" ] && opt=":${v#*:}"
  libs="$libs $V/librasr_gmm_$name.so$opt"
done
timeout -k 10 300 python scripts/ab_bench.py --mode $mode --rounds 2 --dim ${DIM:-39} $libs
