#!/bin/bash
# kernel profiles at the new default micro-batch (512): steady-state micro-step + whole bench.py run
mkdir -p gpurun_out
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/s3_prof512 -o albert --output-format csv -- python bench/model_step.py --impl dedloc --batch 512 --iters 3 --warmup 2 > gpurun_out/s3_prof512.log 2>&1
rc=$?; echo rc=$rc; grep '^{' gpurun_out/s3_prof512.log | cut -c1-200
[ $rc -ne 0 ] && exit $rc
python scripts/trace_tail_stats.py gpurun_out/s3_prof512/albert_kernel_trace.csv gpurun_out/s3_prof512/albert_b512_steady_stats.csv --window 1.1 --skip_tail 0.0
rm -f gpurun_out/s3_prof512/*kernel_trace.csv
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/s3_profbench -o bench --output-format csv -- python bench.py --steps 1 --warmup 1 > gpurun_out/s3_profbench.log 2>&1
rc=$?; echo rc=$rc; grep '^{' gpurun_out/s3_profbench.log | cut -c1-300
rm -f gpurun_out/s3_profbench/*kernel_trace.csv
[ $rc -ne 0 ] && exit $rc
# BASELINE config 3: collaborative SwAV peer (target 32768 samples per collaborative step)
timeout -k 10 600 python -u bench.py --model swav --steps 2 --warmup 1 > gpurun_out/s3_swav_bench.log 2>&1
rc=$?; echo rc=$rc; grep '^{' gpurun_out/s3_swav_bench.log | cut -c1-400; [ $rc -ne 0 ] && tail -20 gpurun_out/s3_swav_bench.log
exit $rc
