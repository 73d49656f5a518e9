#!/bin/bash
# Fail-fast GPU pass: stop at the first timeout/abort/segfault (rc >= 124); test failures (rc 1) continue.
mkdir -p gpurun_out
export PYTHONPATH=$PWD
step() {
  local log=$1; shift
  timeout -k 10 "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"; tail -3 "$log"
  if [ $rc -ge 124 ]; then echo "stopping after rc=$rc"; exit $rc; fi
}
step gpurun_out/pytest_gpu.log 900 python -m pytest tests -q -m gpu
step gpurun_out/swav_step.log 600 python bench/swav_step.py --batch 64 --iters 8
step gpurun_out/swav_step_grouped.log 600 python bench/swav_step.py --batch 64 --iters 8 --grouped --queue
step gpurun_out/step_dedloc5.log 300 python bench/model_step.py --impl dedloc --batch 64 --iters 5
step gpurun_out/bench5.log 900 python bench.py --micro_batch 64
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step gpurun_out/prof5.log 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_step5 -o step --output-format csv -- python bench/model_step.py --impl dedloc --batch 64 --iters 3 --warmup 2
step gpurun_out/profswav5.log 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_swav5 -o swav --output-format csv -- python bench/swav_step.py --batch 64 --iters 3 --warmup 2
