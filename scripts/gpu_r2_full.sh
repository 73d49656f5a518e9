#!/bin/bash
# full GPU tier + smoke + 1-GPU bench (round-end rehearsal)
mkdir -p gpurun_out
export PYTHONPATH=$PWD
step() {
  local log=$1; shift
  timeout -k 10 "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"; grep -E '^\{|passed|failed|Error' "$log" | tail -12 | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; tail -40 "$log"; exit $rc; fi
}
step gpurun_out/full_pytest.log 900 python -u -m pytest tests -q -m gpu -x --timeout 240 --timeout-method thread
step gpurun_out/full_smoke.log 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step gpurun_out/full_bench.log 600 python bench.py
