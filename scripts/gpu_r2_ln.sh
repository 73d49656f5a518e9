#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
step() {
  local log=$1; shift
  timeout -k 10 "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"; grep -E '^\{|passed|failed|Error' "$log" | tail -12 | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; tail -40 "$log"; exit $rc; fi
}
step gpurun_out/ln_pytest.log 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "layernorm or ln or albert" --timeout 120 --timeout-method thread
step gpurun_out/ln_ew.log 300 python -u bench/ew_bench.py
step gpurun_out/ln_step.log 400 python -u bench/model_step.py --impl dedloc --batch 256 --iters 6 --warmup 3
