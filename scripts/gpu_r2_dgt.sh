#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
T=131072 DGRAD_T=1 VARIANTS=lt timeout -k 10 300 python -u bench/gemm_bench.py --check > gpurun_out/dgt.log 2>&1; rc=$?
echo rc=$rc; grep '^{' gpurun_out/dgt.log | cut -c1-300
