#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
for B in 64 128 256; do
timeout -k 10 300 python -u bench/model_step.py --impl dedloc --batch $B --iters 8 --warmup 3 > gpurun_out/mb_$B.log 2>&1 || exit 1
grep '^{' gpurun_out/mb_$B.log | cut -c1-200
done
