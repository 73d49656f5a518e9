# gemm8 DMUL epilogue: packed product stored directly (in-tree) vs HEAD
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels_fuzz_gpu.py tests/test_swav_kernels_gpu.py > gpurun_out/dm_t.log 2>&1 || { tail -40 gpurun_out/dm_t.log; exit 1; }
tail -1 gpurun_out/dm_t.log
timeout -k 10 600 python bench/ab_native.py --lib ab/_C_base.so --rounds 2 --timeout 280 -- env T=262144 python bench/gemm_bench.py > gpurun_out/dm_gemm_ab.jsonl 2>&1 || { tail -20 gpurun_out/dm_gemm_ab.jsonl; exit 1; }
timeout -k 10 900 python bench/ab_native.py --lib ab/_C_base.so --rounds 3 --timeout 280 -- python bench/model_step.py --batch 512 --iters 6 --warmup 2 > gpurun_out/dm_step_ab.jsonl 2>&1 || { tail -20 gpurun_out/dm_step_ab.jsonl; exit 1; }
cat gpurun_out/dm_step_ab.jsonl
