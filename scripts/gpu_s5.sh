#!/bin/bash
# ALBERT micro-batch sweep (global batch fixed at 4096 samples per collaborative step)
mkdir -p gpurun_out
export PYTHONPATH=$PWD
for mb in 128 256 64; do
  timeout -k 10 400 python bench.py --micro_batch $mb > gpurun_out/s5_bench_mb$mb.log 2>&1
  rc=$?; echo "mb=$mb rc=$rc"; grep '^{' gpurun_out/s5_bench_mb$mb.log | cut -c1-260
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/s5_bench_mb$mb.log; exit $rc; fi
done
