# SwAV b=64 iteration: gemm8 epilogue addressing (in-tree) vs previous commit (ab/_C_base.so)
set -e
mkdir -p gpurun_out
timeout -k 10 900 python bench/ab_native.py --lib ab/_C_base.so --rounds 3 --timeout 280 -- python bench/swav_step.py --graph --iters 30 > gpurun_out/swav_epi_ab.jsonl 2>&1 || { tail -20 gpurun_out/swav_epi_ab.jsonl; exit 1; }
cat gpurun_out/swav_epi_ab.jsonl
