#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
T=131072 VARIANTS=lt timeout -k 10 300 python -u bench/gemm_bench.py > gpurun_out/tune64.log 2>&1; echo rc=$?
T=131072 VARIANTS=lt DEDLOC_LT_TUNE=1024 timeout -k 10 600 python -u bench/gemm_bench.py > gpurun_out/tune1024.log 2>&1; echo rc=$?
DEDLOC_LT_DEBUG=1 T=131072 VARIANTS=lt DEDLOC_LT_TUNE=1024 timeout -k 10 300 python -u -c "
import os, torch, dedloc_amd.ops
O=torch.ops.dedloc
dy=torch.randn(131072,4096,device='cuda').bfloat16(); x=torch.randn(131072,1024,device='cuda').bfloat16()
g=torch.zeros(4096,1024,device='cuda'); O.gemm_acc_f32(dy,x,g,True,False); torch.cuda.synchronize()
" > gpurun_out/tune_dbg.log 2>&1; echo rc=$?
paste <(grep -o '"gemm": "[^"]*"\|"lt_us": [0-9.]*' gpurun_out/tune64.log | paste - - ) <(grep -o '"lt_us": [0-9.]*' gpurun_out/tune1024.log)
grep "\[lt\]" gpurun_out/tune_dbg.log | head
