#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
T=131072 DGRAD_T=1 VARIANTS=gemm8,lt timeout -k 10 400 python -u bench/gemm_bench.py --check > gpurun_out/g8dg.log 2>&1; rc=$?
echo rc=$rc; grep '^{' gpurun_out/g8dg.log | grep -v '"check"' | cut -c1-200; grep '"check"' gpurun_out/g8dg.log | grep dgelu | cut -c1-200
