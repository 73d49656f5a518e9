#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_alb -o step --output-format csv -- python bench/model_step.py --impl dedloc --batch 64 --iters 4 --warmup 3 > gpurun_out/prof_alb.log 2>&1; echo rc=$?
python scripts/trace_tail_stats.py gpurun_out/prof_alb/step_kernel_trace.csv gpurun_out/prof_alb/step_steady_stats.csv --window 0.3 && rm -f gpurun_out/prof_alb/*kernel_trace.csv
