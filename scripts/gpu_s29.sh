#!/bin/bash
# LayerNorm-backward grid cap A/B (model step B=64 and B=256)
export PYTHONPATH=$PWD
for p in 512 768 1024; do
  for b in 64 256; do
    it=$([ $b = 64 ] && echo 12 || echo 4)
    DEDLOC_LN_PARTS=$p timeout -k 10 300 python bench/model_step.py --impl dedloc --batch $b --iters $it --warmup 3 > gpurun_out/s29_${p}_${b}.log 2>&1 || exit 1
    echo "parts=$p B=$b $(grep '^{' gpurun_out/s29_${p}_${b}.log | cut -c1-120)"
  done
done
