#!/bin/bash
# GPU multi-crop augmentation kernels: numerics vs reference, SwAV step with the kernel data path
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_swav.py -x -q --timeout 120 --timeout-method thread -m gpu \
  > gpurun_out/s15_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s15_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench/swav_step.py --batch 64 --iters 20 2>&1 | tee gpurun_out/s15_swav.log | grep -E '^\{|warmup 0'
