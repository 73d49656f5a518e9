#!/bin/bash
# Same-box A/B of the ALBERT-large B=512 micro-step: runs bench/model_step.py once per
# "ENV=VALUE" argument (or "base" for no change), twice each, interleaved.
# usage: bash scripts/ab_model_step.sh OUTFILE base DEDLOC_GEMM8_GROUP=1
set -o pipefail
out=$1; shift
for round in 1 2; do
  for arm in "$@"; do
    if [ "$arm" = base ]; then envs=(); else envs=("$arm"); fi
    echo "arm=$arm round=$round" >> "$out"
    env "${envs[@]}" timeout -k 10 240 python -u bench/model_step.py --batch 512 --iters 6 --warmup 2 2>/dev/null | grep samples_per_s >> "$out" || exit 1
  done
done
