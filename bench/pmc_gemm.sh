#!/bin/bash
# PMC passes over single GEMM kinds (bench/gemm_one.py): main-loop anatomy of gemm8 per operand
# layout.  usage: bash bench/pmc_gemm.sh OUTDIR "gemm:kind" ...
repo=$(cd "$(dirname "$0")/.." && pwd)
out=$(cd "$1" 2>/dev/null && pwd || (mkdir -p "$1" && cd "$1" && pwd)); shift
cd /tmp && export TMPDIR=/tmp
PA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
PB="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
PC="FETCH_SIZE SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
for gk in "$@"; do
  g=${gk%%:*}; k=${gk#*:}
  for pass in A B C; do
    if [ $pass = A ]; then ctr=$PA; elif [ $pass = B ]; then ctr=$PB; else ctr=$PC; fi
    timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d $out/${g}_${k}_$pass -o p -- \
      python3 $repo/bench/gemm_one.py --gemm $g --kind $k --iters 5 || exit $?
  done
done
