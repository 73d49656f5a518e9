#!/bin/bash
# Round-2 steady-state kernel profile of the ALBERT-large micro-step at B=256
mkdir -p gpurun_out
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r2_prof -o albert --output-format csv -- python bench/model_step.py --impl dedloc --batch 256 --iters 4 --warmup 2 > gpurun_out/r2_prof.log 2>&1
rc=$?; echo rc=$rc; tail -3 gpurun_out/r2_prof.log | cut -c1-300
[ $rc -ne 0 ] && exit $rc
python scripts/trace_tail_stats.py gpurun_out/r2_prof/albert_kernel_trace.csv gpurun_out/r2_prof/albert_b256_steady_stats.csv --window 0.9 --skip_tail 0.0
rm -f gpurun_out/r2_prof/*kernel_trace.csv
