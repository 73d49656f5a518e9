#!/bin/bash
# Session-2: conv kernel numerics + per-shape bench vs MIOpen, full GPU tests, smoke, headline bench,
# SwAV iteration (hip conv vs MIOpen) and a steady-state kernel profile of the SwAV iteration.
mkdir -p gpurun_out
export PYTHONPATH=$PWD
step() {
  local log=$1; shift
  timeout -k 10 "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"; grep -E '^\{|passed|failed' "$log" | tail -60 || tail -4 "$log"
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; tail -30 "$log"; exit $rc; fi
}
step gpurun_out/s2_conv_tests.log 300 python -u -m pytest tests/test_conv.py -x -q -m gpu --timeout 120 --timeout-method thread
step gpurun_out/s2_conv_bench.log 400 python bench/conv_bench.py
step gpurun_out/s2_swav_hip.log 300 python bench/swav_step.py --batch 64 --iters 10
DEDLOC_CONV=miopen step gpurun_out/s2_swav_miopen.log 300 python bench/swav_step.py --batch 64 --iters 10
step gpurun_out/s2_pytest.log 900 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread
step gpurun_out/s2_smoke.log 300 python __graft_entry__.py smoke
step gpurun_out/s2_bench.log 600 python bench.py
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step gpurun_out/s2_swavprof.log 600 rocprofv3 --kernel-trace --stats -d gpurun_out/s2_prof_swav -o swav --output-format csv -- python bench/swav_step.py --batch 64 --iters 20 --warmup 6
python scripts/trace_tail_stats.py gpurun_out/s2_prof_swav/swav_kernel_trace.csv gpurun_out/s2_prof_swav/swav_steady_stats.csv --window 0.6 --skip_tail 0.3
rm -f gpurun_out/s2_prof_swav/*kernel_trace.csv
