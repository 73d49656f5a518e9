#!/bin/bash
# power / clock while the ALBERT micro-step runs (is the GEMM-heavy step power-bound?)
mkdir -p gpurun_out
export PYTHONPATH=$PWD
( for i in $(seq 1 40); do date +%s.%N; timeout 10 rocm-smi --showpower --showclocks --showtemp 2>/dev/null | grep -E "Power|sclk|mclk|Temperature" ; sleep 1; done ) > gpurun_out/power_samples.txt 2>&1 &
SMI=$!
timeout -k 10 240 python -u bench/model_step.py --impl dedloc --batch 512 --iters 40 --warmup 2 > gpurun_out/power_step.log 2>&1
rc=$?
kill $SMI 2>/dev/null; wait $SMI 2>/dev/null
grep '^{' gpurun_out/power_step.log | cut -c1-200
grep -E "Power|sclk" gpurun_out/power_samples.txt | sort | uniq -c | sort -rn | head -20
exit $rc
