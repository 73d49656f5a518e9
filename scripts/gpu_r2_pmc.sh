#!/bin/bash
# PMC passes over the attention kernels (one counter group per run, --kernel-trace only)
mkdir -p gpurun_out/pmc
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1; echo "list rc=$?"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d gpurun_out/pmc/p$i -o attn --output-format csv -- python bench/attn_pmc.py > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; tail -2 gpurun_out/pmc/p$i.log | cut -c1-300
  [ $rc -ne 0 ] && exit $rc
done
exit 0
