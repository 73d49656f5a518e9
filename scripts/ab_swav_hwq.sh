#!/bin/bash
# HW-queue count vs SwAV concurrent pass splits (same box, interleaved)
out=gpurun_out/r4_swav_hwq.txt
for round in 1 2; do
  for q in 4 8; do
    for sp in 2,1 2,2; do
      echo "hwq=$q splits=$sp round=$round" >> $out
      GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python -u bench/swav_step.py --graph --iters 30 --splits $sp 2>/dev/null | tail -1 >> $out || exit 1
    done
  done
done
