#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/smoke.log
for b in 32 64; do timeout -k 10 300 python bench/model_step.py --impl dedloc --batch $b --iters 6 >> gpurun_out/step_dedloc.log 2>&1 || exit 1; done
tail -2 gpurun_out/step_dedloc.log
timeout -k 10 300 python bench/model_step.py --impl hf --batch 32 --iters 6 --with_optimizer > gpurun_out/step_hf_opt.log 2>&1; tail -1 gpurun_out/step_hf_opt.log
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --verbose > gpurun_out/bench1.log 2>&1; echo "bench rc=$?"; grep metric gpurun_out/bench1.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_step2 -o step --output-format csv -- python bench/model_step.py --impl dedloc --batch 32 --iters 3 --warmup 2 > gpurun_out/prof2.log 2>&1; echo "prof rc=$?"
