#!/bin/bash
# ALBERT headline bench (auto micro-batch) + steady-state kernel profile of the micro-step at B=256
mkdir -p gpurun_out
export PYTHONPATH=$PWD
step() {
  local log=$1; shift
  timeout -k 10 "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"; grep -E '^\{|passed|failed|window' "$log" | tail -5 | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; tail -30 "$log"; exit $rc; fi
}
step gpurun_out/s6_bench.log 600 python bench.py
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step gpurun_out/s6_prof.log 600 rocprofv3 --kernel-trace --stats -d gpurun_out/s6_prof_albert -o albert --output-format csv -- python bench/model_step.py --impl dedloc --batch 256 --iters 4 --warmup 2
python scripts/trace_tail_stats.py gpurun_out/s6_prof_albert/albert_kernel_trace.csv gpurun_out/s6_prof_albert/albert_b256_steady_stats.csv --window 0.9 --skip_tail 0.0
rm -f gpurun_out/s6_prof_albert/*kernel_trace.csv
