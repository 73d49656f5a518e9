#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; grep -E "passed|failed|Error|assert" gpurun_out/pytest_gpu.log | head -20
timeout -k 10 300 python bench/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1; echo "gemm rc=$?"; cat gpurun_out/gemm_bench.log | tail -14
for b in 64; do timeout -k 10 300 python bench/model_step.py --impl dedloc --batch $b --iters 5 >> gpurun_out/step_dedloc4.log 2>&1; done; grep impl gpurun_out/step_dedloc4.log
DEDLOC_GEMM=lib timeout -k 10 300 python bench/model_step.py --impl dedloc --batch 64 --iters 5 >> gpurun_out/step_dedloc4.log 2>&1; grep impl gpurun_out/step_dedloc4.log | tail -1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_step4 -o step --output-format csv -- python bench/model_step.py --impl dedloc --batch 64 --iters 3 --warmup 2 > gpurun_out/prof4.log 2>&1; echo "prof rc=$?"
