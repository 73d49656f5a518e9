#!/bin/bash
# conv v3: persistent multi-tile forward + row-padded stem im2col
mkdir -p gpurun_out
export PYTHONPATH=$PWD
step() {
  local log=$1; shift
  timeout -k 10 "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"; grep -E '^\{"total|^\{"metric|passed|failed' "$log" | tail -20 || tail -4 "$log"
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; tail -30 "$log"; exit $rc; fi
}
step gpurun_out/s4_conv_tests.log 300 python -u -m pytest tests/test_conv.py -x -q -m gpu --timeout 120 --timeout-method thread
step gpurun_out/s4_conv_bench.log 400 python bench/conv_bench.py
step gpurun_out/s4_swav_hip.log 300 python bench/swav_step.py --batch 64 --iters 10
WGRAD_QUICK=1 step gpurun_out/s4_wgrad.log 300 python bench/wgrad_bench.py
step gpurun_out/s4_bench.log 600 python bench.py
