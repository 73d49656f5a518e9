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
step gpurun_out/cvt_pytest.log 900 python -u -m pytest tests -q -m gpu -x --timeout 240 --timeout-method thread
step gpurun_out/cvt_ew.log 300 python -u bench/ew_bench.py
step gpurun_out/cvt_attn.log 300 python -u bench/attn_bench.py --batch 256
step gpurun_out/cvt_step.log 400 python -u bench/model_step.py --impl dedloc --batch 256 --iters 6 --warmup 3
step gpurun_out/cvt_bench.log 600 python bench.py
