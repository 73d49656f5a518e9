#!/bin/bash
# PMC passes over the SwAV b=64 iteration (bench/swav_step.py, eager launches, 3 timed iterations)
repo=$(cd "$(dirname "$0")/.." && pwd)
out=$(mkdir -p "$1" && cd "$1" && pwd)
cd /tmp && export TMPDIR=/tmp
PA="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
PB="FETCH_SIZE GRBM_GUI_ACTIVE"
PC="WRITE_SIZE GRBM_GUI_ACTIVE"
for pass in A B C; do
  if [ $pass = A ]; then ctr=$PA; elif [ $pass = B ]; then ctr=$PB; else ctr=$PC; fi
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d $out/$pass -o p -- \
    python3 $repo/bench/swav_step.py --iters 3 --warmup 2 || exit $?
  echo "pass $pass done"
done
