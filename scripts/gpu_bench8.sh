#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -m gpu -k attention > gpurun_out/pytest_attn3.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_attn3.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 120 python bench/attn_bench.py || exit $?
timeout -k 10 600 python bench/wgrad_bench.py
