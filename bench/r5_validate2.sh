set -e
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_r5c.log 2>&1 || { tail -20 gpurun_out/bench_r5c.log; exit 1; }
tail -1 gpurun_out/bench_r5c.log | cut -c1-200
timeout -k 10 600 python bench.py --model swav > gpurun_out/bench_swav_r5c.log 2>&1 || { tail -20 gpurun_out/bench_swav_r5c.log; exit 1; }
tail -1 gpurun_out/bench_swav_r5c.log | cut -c1-200
