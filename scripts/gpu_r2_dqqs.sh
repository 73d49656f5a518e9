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
step gpurun_out/dqqs_pytest.log 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "attn or attention" --timeout 120 --timeout-method thread
DEDLOC_ATTN_DQ_QS=1 step gpurun_out/dqqs_b1.log 300 python -u bench/attn_bench.py --batch 256
step gpurun_out/dqqs_b2.log 300 python -u bench/attn_bench.py --batch 256
DEDLOC_ATTN_DQ_QS=1 step gpurun_out/dqqs_b1b.log 300 python -u bench/attn_bench.py --batch 256
step gpurun_out/dqqs_b2b.log 300 python -u bench/attn_bench.py --batch 256
DEDLOC_ATTN_RING=0 step gpurun_out/dqqs_b2r0.log 300 python -u bench/attn_bench.py --batch 256
