#!/bin/bash
mkdir -p gpurun_out/pmc_g8
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P -d gpurun_out/pmc_g8/p$i -o g8 --output-format csv -- python bench/gemm8_pmc.py > gpurun_out/pmc_g8/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && tail -5 gpurun_out/pmc_g8/p$i.log && exit $rc
done
python scripts/pmc_summary.py gemm8 gpurun_out/pmc_g8/p1/g8_counter_collection.csv gpurun_out/pmc_g8/p2/g8_counter_collection.csv
exit 0
