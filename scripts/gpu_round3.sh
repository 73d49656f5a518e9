#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/pytest_gpu.log
for b in 32 64 128; do timeout -k 10 300 python bench/model_step.py --impl dedloc --batch $b --iters 5 >> gpurun_out/step_dedloc3.log 2>&1 || exit 1; done
grep impl gpurun_out/step_dedloc3.log
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --micro_batch 64 > gpurun_out/bench3.log 2>&1; echo "bench rc=$?"; grep metric gpurun_out/bench3.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_step3 -o step --output-format csv -- python bench/model_step.py --impl dedloc --batch 64 --iters 3 --warmup 2 > gpurun_out/prof3.log 2>&1; echo "prof rc=$?"
