#!/bin/bash
# Same-box A/B of two source trees (Python-level changes): arm A = ./ab_old (a git worktree of the
# previous commit with this tree's built libraries copied in), arm B = this tree.
# usage: bash scripts/ab_swav_trees.sh OUTFILE [swav_step args...]
set -o pipefail
out=$1; shift
for round in ${ROUNDS:-1 2 3}; do
  for arm in A B; do
    dir=.; [ $arm = A ] && dir=ab_old
    echo "arm=$arm round=$round" >> "$out"
    (cd $dir && timeout -k 10 240 python -u bench/swav_step.py "$@" 2>/dev/null | tail -1) >> "$out" || exit 1
  done
done
