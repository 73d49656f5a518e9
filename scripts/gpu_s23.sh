#!/bin/bash
# conv backend: per-shape auto (MIOpen for the stem and the 64-channel 3x3 convs) vs hip + MIOpen stem
mkdir -p gpurun_out
export PYTHONPATH=$PWD
for cfg in "--conv auto --stem null" "--conv hip"; do
  tag=$(echo $cfg | tr -d ' -')
  timeout -k 10 300 python bench/swav_step.py --batch 64 --iters 30 $cfg 2>&1 | tee gpurun_out/s23_$tag.log | grep -E '^\{|warmup 0' | cut -c1-200
  rc=${PIPESTATUS[0]}; echo "cfg=$cfg rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
