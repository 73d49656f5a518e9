#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r2_swav -o swav --output-format csv -- python bench/swav_step.py --batch 64 --iters 12 > gpurun_out/r2_swav.log 2>&1
rc=$?; echo rc=$rc; grep '^{' gpurun_out/r2_swav.log | cut -c1-200
[ $rc -ne 0 ] && exit $rc
python scripts/trace_tail_stats.py gpurun_out/r2_swav/swav_kernel_trace.csv gpurun_out/r2_swav/swav_steady_stats.csv --window 0.25 --skip_tail 0.0
rm -f gpurun_out/r2_swav/*kernel_trace.csv
