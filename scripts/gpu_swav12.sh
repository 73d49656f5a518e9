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
step gpurun_out/pytest_swav12.log 600 python -m pytest tests/test_swav.py -q -m gpu
step gpurun_out/swav12_graph.log 600 python bench/swav_step.py --batch 64 --iters 10
step gpurun_out/swav12_eager.log 600 python bench/swav_step.py --batch 64 --iters 10 --no_graph
step gpurun_out/swav12_grouped.log 600 python bench/swav_step.py --batch 64 --iters 10 --grouped
