#!/bin/bash
# Session-2 validation: full GPU test tier, smoke, headline bench, SwAV step (default backend + data kernels)
mkdir -p gpurun_out
export PYTHONPATH=$PWD
step() {
  local log=$1; shift
  timeout -k 10 "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"; grep -E '^\{|passed|failed|smoke' "$log" | tail -5 | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; tail -30 "$log"; exit $rc; fi
}
step gpurun_out/s18_pytest.log 900 python -u -m pytest tests -q -m gpu --timeout 240 --timeout-method thread
step gpurun_out/s18_smoke.log 300 python __graft_entry__.py smoke
step gpurun_out/s18_bench.log 600 python bench.py
step gpurun_out/s18_swav.log 300 python bench/swav_step.py --batch 64 --iters 20
