# (2,1) concurrent-pass default: SwAV tests, the SwAV bench.py line, swav_step default vs --splits 1,1
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_swav.py tests/test_swav_parity_gpu.py tests/test_swav_kernels_gpu.py > gpurun_out/spc_t.log 2>&1 || { tail -40 gpurun_out/spc_t.log; exit 1; }
tail -1 gpurun_out/spc_t.log
timeout -k 10 600 python bench.py --model swav > gpurun_out/spc_bench_swav.log 2>&1 || { tail -20 gpurun_out/spc_bench_swav.log; exit 1; }
tail -1 gpurun_out/spc_bench_swav.log | cut -c1-220
for r in 1 2; do
  for sp in default 1,1; do
    if [ $sp = default ]; then a=""; else a="--splits $sp"; fi
    timeout -k 10 280 python bench/swav_step.py --graph --iters 30 $a > gpurun_out/spc_$sp.$r.log 2>&1 || { tail -20 gpurun_out/spc_$sp.$r.log; exit 1; }
    echo "splits $sp round $r $(grep -o '"value": [0-9.]*' gpurun_out/spc_$sp.$r.log)"
  done
done
