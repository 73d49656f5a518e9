#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -m gpu -x -k "layernorm or albert" --timeout 120 --timeout-method thread > gpurun_out/lnw_pytest.log 2>&1; rc=$?; tail -1 gpurun_out/lnw_pytest.log; [ $rc -ne 0 ] && exit $rc
for T in 32768 131072; do
for W in 4 8; do
T=$T DEDLOC_LN_WPB=$W timeout -k 10 120 python -u bench/ew_bench.py > gpurun_out/lnw_${T}_$W.log 2>&1 || exit 1
echo "T=$T wpb=$W $(grep ln_bwd gpurun_out/lnw_${T}_$W.log | cut -c1-120)"
done
done
