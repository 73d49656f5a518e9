#!/bin/bash
# steady-state kernel profile of the ALBERT micro-step at B=256 (after the attention XCD order)
mkdir -p gpurun_out
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/s26_prof_albert -o albert --output-format csv -- python bench/model_step.py --impl dedloc --batch 64 --iters 12 --warmup 4 > gpurun_out/s26_prof.log 2>&1
rc=$?; grep '^{' gpurun_out/s26_prof.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
python scripts/trace_tail_stats.py gpurun_out/s26_prof_albert/albert_kernel_trace.csv gpurun_out/s26_prof_albert/albert_b64_steady_stats.csv --window 0.9 --skip_tail 0.0
rm -f gpurun_out/s26_prof_albert/*kernel_trace.csv
