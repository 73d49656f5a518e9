#!/bin/bash
# Round-2 checkpoint: GPU test tier, smoke, headline bench (fail-fast on any non-zero exit).
mkdir -p gpurun_out
export PYTHONPATH=$PWD
step() {
  local log=$1; shift
  timeout -k 10 "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"; grep -E '^\{|passed|failed|smoke' "$log" | tail -5 | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; tail -30 "$log"; exit $rc; fi
}
step gpurun_out/r2_pytest.log 900 python -u -m pytest tests -q -m gpu -x --timeout 240 --timeout-method thread
step gpurun_out/r2_smoke.log 300 python __graft_entry__.py smoke
step gpurun_out/r2_bench.log 600 python bench.py
