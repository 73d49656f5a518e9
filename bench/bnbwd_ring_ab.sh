# gemm8 BN-backward epilogue: R / X / Y on one read-ahead ring (in-tree RD=3, ab/_C_rd4.so RD=4) vs HEAD
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_swav_kernels_gpu.py tests/test_conv.py > gpurun_out/br_t.log 2>&1 || { tail -40 gpurun_out/br_t.log; exit 1; }
tail -1 gpurun_out/br_t.log
timeout -k 10 1000 python bench/ab_native.py --lib ab/_C_base.so --rounds 3 --timeout 280 -- python bench/swav_step.py --graph --iters 30 > gpurun_out/br_swav_ab.jsonl 2>&1 || { tail -20 gpurun_out/br_swav_ab.jsonl; exit 1; }
python3 scripts/ab_summary.py gpurun_out/br_swav_ab.jsonl
timeout -k 10 1000 python bench/ab_native.py --lib ab/_C_rd4.so --rounds 3 --timeout 280 -- python bench/swav_step.py --graph --iters 30 > gpurun_out/br_swav_ab_rd4.jsonl 2>&1 || { tail -20 gpurun_out/br_swav_ab_rd4.jsonl; exit 1; }
python3 scripts/ab_summary.py gpurun_out/br_swav_ab_rd4.jsonl
