#!/bin/bash
# two-round hipBLASLt autotune: GEMM numerics, then the headline bench twice (variance check)
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu \
  > gpurun_out/s25_tests.log 2>&1; rc=$?; tail -1 gpurun_out/s25_tests.log; [ $rc -ne 0 ] && exit $rc
for k in 1 2; do
  timeout -k 10 600 python bench.py > gpurun_out/s25_bench_$k.log 2>&1; rc=$?; grep '^{' gpurun_out/s25_bench_$k.log | cut -c1-180; [ $rc -ne 0 ] && exit $rc
done
exit 0
