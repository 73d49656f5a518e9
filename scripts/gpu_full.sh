#!/bin/bash
# Full GPU confirmation pass: pytest -m gpu, smoke, bench.py (fail-fast on timeouts/aborts).
mkdir -p gpurun_out
export PYTHONPATH=$PWD
step() {
  local log=$1; shift
  timeout -k 10 "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"; grep -E '^\{|passed|failed|smoke ok' "$log" | tail -3
  if [ $rc -ge 124 ]; then echo "stopping after rc=$rc"; exit $rc; fi
}
step gpurun_out/full_pytest.log 1200 python -m pytest tests -q -m gpu
grep FAILED gpurun_out/full_pytest.log | head
step gpurun_out/full_smoke.log 300 python -c "import __graft_entry__ as g; g.smoke()"
step gpurun_out/full_bench.log 900 python bench.py
