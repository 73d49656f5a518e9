#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
step() {
  local log=$1; shift
  timeout -k 10 "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"; tail -4 "$log"
  if [ $rc -ge 124 ]; then echo "stopping after rc=$rc"; exit $rc; fi
}
step gpurun_out/lt_debug7.log 300 python scripts/lt_debug.py
step gpurun_out/pytest_gpu7.log 900 python -m pytest tests -q -m gpu
grep -E "passed|failed|FAILED" gpurun_out/pytest_gpu7.log | tail -15
step gpurun_out/step7.log 300 python bench/model_step.py --impl dedloc --batch 64 --iters 5
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step gpurun_out/prof7.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_step7 -o step --output-format csv -- python bench/model_step.py --impl dedloc --batch 64 --iters 3 --warmup 2
