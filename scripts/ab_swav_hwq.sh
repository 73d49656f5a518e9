#!/bin/bash
# HW-queue count for the SwAV iteration (same box, interleaved): GPU_MAX_HW_QUEUES in ${QUEUES:-4 8}
out=${OUT:-gpurun_out/r4_swav_hwq.txt}
for round in ${ROUNDS:-1 2}; do
  for q in ${QUEUES:-4 8}; do
    echo "hwq=$q round=$round" >> $out
    GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python -u bench/swav_step.py --graph --iters 40 2>/dev/null | tail -1 >> $out || exit 1
  done
done
