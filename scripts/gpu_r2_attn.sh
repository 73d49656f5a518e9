#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
step() {
  local log=$1; shift
  timeout -k 10 "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"; grep -E '^\{|passed|failed|Error' "$log" | tail -12 | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; tail -40 "$log"; exit $rc; fi
}
step gpurun_out/at_pytest.log 600 python -u -m pytest tests -q -m gpu -x --timeout 240 --timeout-method thread
step gpurun_out/at_bench.log 600 python bench.py
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step gpurun_out/at_prof.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b256 -o step --output-format csv -- python bench/model_step.py --impl dedloc --batch 256 --iters 3 --warmup 2
