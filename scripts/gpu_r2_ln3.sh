#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
for i in 1 2; do
for R in 2 4; do
DEDLOC_LN_ROWS=$R timeout -k 10 300 python -u bench/ew_bench.py > gpurun_out/ln3_r${R}_$i.log 2>&1 || exit 1
grep ln_bwd gpurun_out/ln3_r${R}_$i.log | cut -c1-200
done
done
DEDLOC_LN_ROWS=4 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "layernorm" --timeout 120 --timeout-method thread 2>&1 | tail -2
