#!/bin/bash
# Same-box A/B of the SwAV b=64 iteration: bench/swav_step.py once per "ENV=VALUE" argument (or
# "base"), twice each, interleaved.  usage: bash scripts/ab_swav_step.sh OUTFILE base DEDLOC_X=0
set -o pipefail
out=$1; shift
for round in 1 2; do
  for arm in "$@"; do
    if [ "$arm" = base ]; then envs=(); else envs=("$arm"); fi
    echo "arm=$arm round=$round" >> "$out"
    env "${envs[@]}" timeout -k 10 240 python -u bench/swav_step.py --iters 20 2>/dev/null | tail -1 >> "$out" || exit 1
  done
done
