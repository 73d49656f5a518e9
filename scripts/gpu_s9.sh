#!/bin/bash
# SwAV step: MIOpen find vs immediate mode vs hand-written convs (progress lines on stderr)
mkdir -p gpurun_out
export PYTHONPATH=$PWD
for cfg in "--conv hip" "--conv miopen --no_find" "--conv miopen"; do
  tag=$(echo $cfg | tr -d ' -')
  timeout -k 10 400 python bench/swav_step.py --batch 64 --iters 10 $cfg 2>&1 | tee gpurun_out/s9_swav_$tag.log | grep -E '^\{|warmup'
  rc=${PIPESTATUS[0]}; echo "cfg=$cfg rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
