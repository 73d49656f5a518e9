#!/bin/bash
# GPU-box checks: kernel tests, model micro-step bench (ours vs HF eager), rocprof kernel stats
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?"
tail -5 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench/model_step.py --impl dedloc --batch 32 > gpurun_out/step_dedloc.log 2>&1 || { echo "dedloc step failed"; tail -20 gpurun_out/step_dedloc.log; exit 1; }
cat gpurun_out/step_dedloc.log | tail -3
timeout -k 10 300 python bench/model_step.py --impl hf --batch 32 > gpurun_out/step_hf.log 2>&1
cat gpurun_out/step_hf.log | tail -3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_step -o step --output-format csv -- python bench/model_step.py --impl dedloc --batch 32 --iters 3 --warmup 2 > gpurun_out/prof.log 2>&1
echo "prof rc=$?"
find gpurun_out/prof_step -name "*stats*" | head
