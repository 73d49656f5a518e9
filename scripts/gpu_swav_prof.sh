#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_swav11 -o swav --output-format csv -- python bench/swav_step.py --batch 64 --iters 20 --warmup 6 > gpurun_out/swav11.log 2>&1; echo rc=$?; python scripts/trace_tail_stats.py gpurun_out/prof_swav11/swav_kernel_trace.csv gpurun_out/prof_swav11/swav_steady_stats.csv --window 0.6 --skip_tail 0.3; rm -f gpurun_out/prof_swav11/*kernel_trace.csv; grep '^{' gpurun_out/swav11.log
