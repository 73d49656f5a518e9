#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u bench/gemm_square.py 2>&1 | tee gpurun_out/gemm_square.log
