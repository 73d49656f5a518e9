# adopted grid sizes (in-tree: BN apply/dx cap 768, wgrad target 192) vs the previous ones (2048 / 256)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv.py tests/test_swav_kernels_gpu.py tests/test_swav.py > gpurun_out/gcc_t.log 2>&1 || { tail -40 gpurun_out/gcc_t.log; exit 1; }
tail -1 gpurun_out/gcc_t.log
timeout -k 10 1200 python bench/ab_native.py --lib ab/_C_old.so --rounds 4 --timeout 280 -- python bench/swav_step.py --graph --iters 30 > gpurun_out/gcc_swav_ab.jsonl 2>&1 || { tail -20 gpurun_out/gcc_swav_ab.jsonl; exit 1; }
python3 scripts/ab_summary.py gpurun_out/gcc_swav_ab.jsonl
