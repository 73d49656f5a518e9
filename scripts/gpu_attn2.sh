#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -m gpu -k attention > gpurun_out/pytest_attn2.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_attn2.log
rc=$?; [ $rc -ge 124 ] && exit $rc
timeout -k 10 120 python bench/attn_bench.py && timeout -k 10 120 python bench/attn_bench.py --pad 0.3
