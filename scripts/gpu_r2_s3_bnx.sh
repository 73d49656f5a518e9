#!/bin/bash
# BN backward ReLU mask from x: SwAV tests + same-box A/B of the b=64 iteration
mkdir -p gpurun_out
export PYTHONPATH=$PWD
step() {
  local log=$1; shift
  timeout -k 10 "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"; grep -E '^\{|passed|failed' "$log" | tail -4 | cut -c1-260
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; tail -30 "$log"; exit $rc; fi
}
step gpurun_out/bnx_pytest.log 400 python -u -m pytest tests/test_swav.py -q -m gpu -x --timeout 200 --timeout-method thread
for r in 1 2; do
  DEDLOC_BN_XMASK=0 step gpurun_out/bnx_off_$r.log 300 python -u bench/swav_step.py --batch 64 --iters 20
  DEDLOC_BN_XMASK=1 step gpurun_out/bnx_on_$r.log 300 python -u bench/swav_step.py --batch 64 --iters 20
done
