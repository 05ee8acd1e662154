#!/bin/bash
# timing only (no correctness check) of library variants: ab_only.sh <mode> v1 v2 ...
V=rasr_amd/lib/variants
mode=$1; shift
libs=""
for v in "$@"; do libs="$libs $V/librasr_gmm_$v.so"; done
timeout -k 10 300 python scripts/ab_bench.py --mode $mode --rounds 2 $libs
