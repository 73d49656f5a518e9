#!/bin/bash
# stem conv backend: hand-written im2col+GEMM vs MIOpen (find mode) for the 3-channel stem only
mkdir -p gpurun_out
export PYTHONPATH=$PWD
for cfg in "--stem miopen" "--stem hip"; do
  tag=$(echo $cfg | tr -d ' -')
  timeout -k 10 300 python bench/swav_step.py --batch 64 --iters 30 $cfg 2>&1 | tee gpurun_out/s17_$tag.log | grep -E '^\{|warmup 0' | cut -c1-220
  rc=${PIPESTATUS[0]}; echo "cfg=$cfg rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
