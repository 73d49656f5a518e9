#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u bench/ew_bench.py 2>&1 | tee gpurun_out/ew_bench.log
