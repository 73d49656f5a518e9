#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
step() {
  local log=$1; shift
  timeout -k 10 "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"; grep -E '^\{|passed|failed|Error' "$log" | tail -12 | cut -c1-250
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; tail -40 "$log"; exit $rc; fi
}
step gpurun_out/wgs_pytest.log 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "albert" --timeout 120 --timeout-method thread
step gpurun_out/wgs_ab256.log 400 python -u bench/ab_step.py --batch 256 --ab wgradstream
step gpurun_out/wgs_ab64.log 400 python -u bench/ab_step.py --batch 64 --ab wgradstream
