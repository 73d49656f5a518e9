#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 ./tests/hip/primitives_test 2>&1 | tee gpurun_out/prim.log
export PYTHONPATH=$PWD
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?"; grep -E "passed|failed|FAILED" gpurun_out/pytest_gpu.log | tail -20
