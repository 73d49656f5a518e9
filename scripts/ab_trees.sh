#!/bin/bash
# Same-box A/B of two source trees on any command: arm A = ./ab_old (a git worktree of an earlier
# commit with this tree's built libraries copied in), arm B = this tree; JSON lines tagged by arm.
# usage: ROUNDS="1 2" bash scripts/ab_trees.sh OUTFILE python bench.py --model swav --steps 2
set -o pipefail
out=$1; shift
for round in ${ROUNDS:-1 2}; do
  for arm in A B; do
    dir=.; [ $arm = A ] && dir=ab_old
    (cd $dir && timeout -k 10 ${LIMIT:-300} "$@" 2>/dev/null | grep '^{' | tail -1 | sed "s/}\$/, \"arm\": \"$arm\", \"round\": $round}/") >> "$out" || exit 1
  done
done
