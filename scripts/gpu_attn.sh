#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
step() {
  local log=$1; shift
  timeout -k 10 "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"; tail -4 "$log"
  if [ $rc -ge 124 ]; then echo "stopping after rc=$rc"; exit $rc; fi
}
step gpurun_out/pytest_attn.log 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -k attention
step gpurun_out/attn_bench.log 120 python bench/attn_bench.py
step gpurun_out/attn_bench_pad.log 120 python bench/attn_bench.py --pad 0.3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step gpurun_out/attn_pmc.log 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/attn_pmc -o attn --output-format csv -- python bench/attn_bench.py --iters 2
step gpurun_out/attn_pmc2.log 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM -d gpurun_out/attn_pmc2 -o attn --output-format csv -- python bench/attn_bench.py --iters 2
