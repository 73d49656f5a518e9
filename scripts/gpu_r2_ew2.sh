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
step gpurun_out/ew2_pytest.log 600 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "gelu or bias or colsum or albert" --timeout 240 --timeout-method thread
step gpurun_out/ew2_bench.log 300 python -u bench/ew_bench.py
step gpurun_out/ew2_ab.log 400 python -u bench/ab_step.py --batch 256 --ab ew
