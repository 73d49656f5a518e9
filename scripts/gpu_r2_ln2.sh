#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
for i in 1 2; do
DEDLOC_LN_ROWS=1 timeout -k 10 300 python -u bench/ew_bench.py > gpurun_out/ln2_r1_$i.log 2>&1 || exit 1
timeout -k 10 300 python -u bench/ew_bench.py > gpurun_out/ln2_r2_$i.log 2>&1 || exit 1
grep ln_bwd gpurun_out/ln2_r1_$i.log gpurun_out/ln2_r2_$i.log | cut -c1-200
done
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "layernorm" --timeout 120 --timeout-method thread 2>&1 | tail -2
