#!/bin/bash
# Fail-fast GPU pass: stop at the first timeout/abort/segfault (rc >= 124); test failures (rc 1) continue.
mkdir -p gpurun_out
export PYTHONPATH=$PWD
step() {
  local log=$1; shift
  timeout -k 10 "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"; tail -4 "$log"
  if [ $rc -ge 124 ]; then echo "stopping after rc=$rc"; exit $rc; fi
}
step gpurun_out/pytest_gpu6.log 900 python -m pytest tests -q -m gpu -x
step gpurun_out/step6_lt.log 300 python bench/model_step.py --impl dedloc --batch 64 --iters 5
DEDLOC_LT=0 step gpurun_out/step6_aten.log 300 python bench/model_step.py --impl dedloc --batch 64 --iters 5
step gpurun_out/bench6.log 900 python bench.py
step gpurun_out/bench6_eager.log 1200 python bench.py --impl eager --steps 2 --warmup 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step gpurun_out/prof6.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_step6 -o step --output-format csv -- python bench/model_step.py --impl dedloc --batch 64 --iters 3 --warmup 2
