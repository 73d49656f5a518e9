#!/bin/bash
# end-of-session validation: GPU tier, smoke, headline bench, SwAV bench
mkdir -p gpurun_out
export PYTHONPATH=$PWD
step() {
  local log=$1; shift
  timeout -k 10 "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"; grep -E '^\{|passed|failed|smoke ok' "$log" | tail -4 | cut -c1-700
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; tail -40 "$log"; exit $rc; fi
}
step gpurun_out/final_pytest.log 900 python -u -m pytest tests -q -m gpu -x --timeout 240 --timeout-method thread
step gpurun_out/final_smoke.log 300 python -c "import __graft_entry__ as g; g.smoke()"
step gpurun_out/final_bench.log 600 python -u bench.py
step gpurun_out/final_bench_swav.log 600 python -u bench.py --model swav --steps 2 --warmup 1
