#!/bin/bash
# plain kernel trace (no counters: concurrent dispatches stay concurrent) of the graphed SwAV b=64 iteration
repo=$(cd "$(dirname "$0")/.." && pwd)
out=$(mkdir -p "$1" && cd "$1" && pwd)
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $out -o kt -- \
  python3 $repo/bench/swav_step.py --graph --iters 6 --warmup 4 > $out/step.log 2>&1 || exit $?
tail -2 $out/step.log
