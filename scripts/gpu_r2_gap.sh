#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
step() {
  local log=$1; shift
  timeout -k 10 "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"; grep -E '^\{|passed|failed|Error' "$log" | tail -12 | cut -c1-600
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; tail -40 "$log"; exit $rc; fi
}
step gpurun_out/gap_step.log 400 python -u bench/model_step.py --impl dedloc --batch 256 --iters 6 --warmup 3
step gpurun_out/gap_bench.log 600 python bench.py --steps 3 --warmup 1 --verbose
