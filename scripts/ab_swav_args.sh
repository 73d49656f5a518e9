#!/bin/bash
# Same-box A/B of bench/swav_step.py argument sets, twice each, interleaved.
# usage: bash scripts/ab_swav_args.sh OUTFILE "" "--sequential" "--graph" ...   ("" = defaults)
set -o pipefail
out=$1; shift
for round in ${ROUNDS:-1 2}; do
  for arm in "$@"; do
    echo "arm=[$arm] round=$round" >> "$out"
    timeout -k 10 240 python -u bench/swav_step.py --iters ${ITERS:-20} $arm 2>/dev/null | tail -1 >> "$out" || exit 1
  done
done
