#!/bin/bash
# PMC passes over the attention kernels (bench/attn_pmc.py: 3 forward + 3 backward calls at
# B x 16 heads x 512 x 64).  usage: bash bench/pmc_attn.sh OUTDIR [B]
repo=$(cd "$(dirname "$0")/.." && pwd)
out=$(mkdir -p "$1" && cd "$1" && pwd)
export B=${2:-512}
cd /tmp && export TMPDIR=/tmp
PA="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"
PB="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE GRBM_COUNT"
PC="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE"
for pass in A B C; do
  if [ $pass = A ]; then ctr=$PA; elif [ $pass = B ]; then ctr=$PB; else ctr=$PC; fi
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d $out/$pass -o p -- \
    python3 $repo/bench/attn_pmc.py || exit $?
done
