#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 500 python -u bench/swav_step.py --batch 64 --iters 10 > gpurun_out/swav_r2.log 2>&1; rc=$?
echo rc=$rc; grep '^{' gpurun_out/swav_r2.log | cut -c1-400; [ $rc -ne 0 ] && tail -20 gpurun_out/swav_r2.log
exit $rc
