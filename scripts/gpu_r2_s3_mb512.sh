#!/bin/bash
# micro-batch 512 (one micro-step per peer per global step at 8 peers): memory + speed vs 256
mkdir -p gpurun_out
export PYTHONPATH=$PWD
step() {
  local log=$1; shift
  timeout -k 10 "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"; grep -E '^\{|Error|error' "$log" | tail -6 | cut -c1-600
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; tail -30 "$log"; exit $rc; fi
}
step gpurun_out/mb512_step.log 300 python -u bench/model_step.py --impl dedloc --batch 512 --iters 6 --warmup 2
step gpurun_out/mb256_step.log 300 python -u bench/model_step.py --impl dedloc --batch 256 --iters 8 --warmup 3
step gpurun_out/mb512_bench.log 600 python -u bench.py --micro_batch 512 --steps 3 --warmup 1
step gpurun_out/mb256_bench.log 600 python -u bench.py --micro_batch 256 --steps 3 --warmup 1
