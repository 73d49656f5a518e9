#!/bin/bash
# conv library routing: kernel tests, per-shape bench, SwAV step with the default (hip) backend
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_conv.py -x -q --timeout 120 --timeout-method thread -m gpu \
  > gpurun_out/s12_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s12_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench/conv_bench.py --batch 64 > gpurun_out/s12_conv_bench.jsonl 2>gpurun_out/s12_conv_bench.err; rc=$?
tail -1 gpurun_out/s12_conv_bench.jsonl; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench/swav_step.py --batch 64 --iters 20 --conv hip 2>&1 | tee gpurun_out/s12_swav.log | grep -E '^\{|warmup'
