#!/bin/bash
# A/B of one library under several values of an environment knob (e.g. RASR_GMM_TARGET_BLOCKS):
#   [AB_ARGS="--frames F --dim D"] scripts/ab_env.sh <mode> <lib> <VAR> <value>...   (each value: its own ab_bench.py run, 2 rounds)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mode=$1; lib=$2; var=$3; shift 3
for v in "$@"; do
  echo "=== $var=$v"
  env "$var=$v" timeout -k 10 300 python scripts/ab_bench.py --mode "$mode" --rounds 2 ${AB_ARGS} "$lib" || exit $?
done
