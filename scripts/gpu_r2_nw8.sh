#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
step() {
  local log=$1; shift
  timeout -k 10 "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"; grep -E '^\{|passed|failed|Error' "$log" | tail -12 | cut -c1-200
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; tail -40 "$log"; exit $rc; fi
}
step gpurun_out/nw8_pytest.log 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "attn or attention" --timeout 120 --timeout-method thread
step gpurun_out/nw8_b4.log 300 python -u bench/attn_bench.py --batch 256
DEDLOC_ATTN_NW=8 step gpurun_out/nw8_b8.log 300 python -u bench/attn_bench.py --batch 256
step gpurun_out/nw8_b4b.log 300 python -u bench/attn_bench.py --batch 256
DEDLOC_ATTN_NW=8 step gpurun_out/nw8_b8b.log 300 python -u bench/attn_bench.py --batch 256
DEDLOC_ATTN_NW=8 step gpurun_out/nw8_b8p.log 300 python -u bench/attn_bench.py --batch 256 --pad 0.3
step gpurun_out/nw8_b4p.log 300 python -u bench/attn_bench.py --batch 256 --pad 0.3
