set -e
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tier_r5f.log 2>&1 || { tail -40 gpurun_out/tier_r5f.log; exit 1; }
tail -1 gpurun_out/tier_r5f.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r5f.log 2>&1 || { tail -20 gpurun_out/smoke_r5f.log; exit 1; }
tail -1 gpurun_out/smoke_r5f.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r5f.log 2>&1 || { tail -20 gpurun_out/bench_r5f.log; exit 1; }
tail -1 gpurun_out/bench_r5f.log | cut -c1-200
timeout -k 10 600 python bench.py --model swav > gpurun_out/bench_swav_r5f.log 2>&1 || { tail -20 gpurun_out/bench_swav_r5f.log; exit 1; }
tail -1 gpurun_out/bench_swav_r5f.log | cut -c1-200
