# gemm8 register-direct epilogue (in-tree _C.so) vs the LDS-staged epilogue (ab/_C_base.so):
# numerics tiers first, then interleaved gemm_bench rounds on the same box.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels_fuzz_gpu.py tests/test_swav_kernels_gpu.py tests/test_conv.py > gpurun_out/gepi_t.log 2>&1 || { tail -40 gpurun_out/gepi_t.log; exit 1; }
tail -2 gpurun_out/gepi_t.log
timeout -k 10 600 python bench/ab_native.py --lib ab/_C_base.so --rounds 2 --timeout 280 -- env T=262144 python bench/gemm_bench.py > gpurun_out/gepi_ab.jsonl 2>&1 || { tail -20 gpurun_out/gepi_ab.jsonl; exit 1; }
echo done
