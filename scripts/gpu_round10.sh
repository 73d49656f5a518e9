#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
step() {
  local log=$1; shift
  timeout -k 10 "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"; tail -4 "$log"
  if [ $rc -ge 124 ]; then echo "stopping after rc=$rc"; exit $rc; fi
}
step gpurun_out/pytest_gpu10.log 900 python -m pytest tests -q -m gpu
grep -E "FAILED" gpurun_out/pytest_gpu10.log | head
step gpurun_out/wgrad10.log 400 python bench/wgrad_bench.py
step gpurun_out/step10.log 300 python bench/model_step.py --impl dedloc --batch 64 --iters 5
step gpurun_out/bench10.log 900 python bench.py
