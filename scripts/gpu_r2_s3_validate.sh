#!/bin/bash
# session-3 re-entry check: GPU tier + headline bench on the restored tree
mkdir -p gpurun_out
export PYTHONPATH=$PWD
step() {
  local log=$1; shift
  timeout -k 10 "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"; grep -E '^\{|passed|failed|Error|RCCL' "$log" | tail -12 | cut -c1-600
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; tail -40 "$log"; exit $rc; fi
}
step gpurun_out/s3_pytest.log 900 python -u -m pytest tests -q -m gpu -x --timeout 240 --timeout-method thread
step gpurun_out/s3_bench.log 600 python bench.py
