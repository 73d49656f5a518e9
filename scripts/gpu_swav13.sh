#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
step() {
  local log=$1; shift
  timeout -k 10 "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"; grep '^{' "$log" || tail -5 "$log"
  if [ $rc -ge 124 ]; then echo "stopping after rc=$rc"; exit $rc; fi
}
step gpurun_out/pytest_swav13.log 600 python -m pytest tests/test_swav.py -q -m gpu
grep -E "FAILED|Error" gpurun_out/pytest_swav13.log | head
step gpurun_out/swav13_eager.log 600 python bench/swav_step.py --batch 64 --iters 10
step gpurun_out/swav13_graph.log 600 python bench/swav_step.py --batch 64 --iters 10 --graph
step gpurun_out/swav13_grouped.log 600 python bench/swav_step.py --batch 64 --iters 10 --grouped
