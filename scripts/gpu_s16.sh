#!/bin/bash
# attention XCD-aware block order: numerics, kernel timing A/B, model step A/B
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "attn or attention" \
  > gpurun_out/s16_tests.log 2>&1; rc=$?; tail -2 gpurun_out/s16_tests.log; [ $rc -ne 0 ] && exit $rc
for x in 0 1; do
  DEDLOC_ATTN_XCD=$x timeout -k 10 300 python bench/attn_bench.py --batch 256 > gpurun_out/s16_attn_$x.log 2>&1; rc=$?; echo "xcd=$x"; tail -3 gpurun_out/s16_attn_$x.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
done
for x in 0 1; do
  DEDLOC_ATTN_XCD=$x timeout -k 10 300 python bench/model_step.py --impl dedloc --batch 256 --iters 6 --warmup 3 > gpurun_out/s16_step_$x.log 2>&1; rc=$?; echo "xcd=$x"; grep '^{' gpurun_out/s16_step_$x.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
done
exit 0
