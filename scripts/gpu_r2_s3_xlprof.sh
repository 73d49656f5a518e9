#!/bin/bash
# albert-xlarge-v2 kernel profile (composed attention share) + whether bmm(out_dtype=fp32) is taken
mkdir -p gpurun_out
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 120 python -c "
import torch; a=torch.randn(4,64,128,device='cuda').bfloat16()
print('bmm out_dtype ok:', torch.bmm(a, a.transpose(1,2), out_dtype=torch.float32).dtype)" 2>&1 | tail -2
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/xlprof -o run -- python3 bench/model_step.py --config albert-xlarge-v2 --batch 64 --iters 3 --warmup 1 > gpurun_out/xlprof.log 2>&1
rc=$?; grep '^{' gpurun_out/xlprof.log | cut -c1-200; exit $rc
