# round-5 session E: end-of-milestone evidence — kernel trace of the B=512 micro-step, the driver's
# 20-step bench, the SwAV bench, the full GPU tier
mkdir -p gpurun_out
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/e_prof -o run -- python bench/model_step.py --batch 512 --iters 4 > gpurun_out/e_prof.log 2>&1
python scripts/rocpd_summary.py $(find gpurun_out/e_prof -name "*results.db" | head -1) --window_ms 1100 > gpurun_out/e_albert_kernels.txt
head -16 gpurun_out/e_albert_kernels.txt
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/e_tier.log 2>&1
tail -1 gpurun_out/e_tier.log
timeout -k 10 500 python bench.py --steps 20 --warmup 1 > gpurun_out/e_bench20.log 2>&1
tail -1 gpurun_out/e_bench20.log
timeout -k 10 500 python bench.py --model swav --steps 3 --warmup 1 > gpurun_out/e_swav.log 2>&1
tail -1 gpurun_out/e_swav.log
