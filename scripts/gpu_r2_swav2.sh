#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
for opt in "" "--grouped" "--graph" "--grouped --graph"; do
timeout -k 10 500 python -u bench/swav_step.py --batch 64 --iters 10 $opt > gpurun_out/swav2.log 2>&1; rc=$?
echo "opt=[$opt] rc=$rc $(grep '^{' gpurun_out/swav2.log | cut -c1-160)"
[ $rc -ne 0 ] && tail -5 gpurun_out/swav2.log
done
exit 0
