#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
step() {
  local log=$1; shift
  timeout -k 10 "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"; grep -E '^\{|passed|failed|Error' "$log" | tail -12 | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; tail -40 "$log"; exit $rc; fi
}
step gpurun_out/wt_pytest.log 600 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x --timeout 240 --timeout-method thread
step gpurun_out/wt_ab.log 600 python -u bench/ab_step.py --batch 256 --ab dgradwt
step gpurun_out/wt_bench.log 600 python bench.py
