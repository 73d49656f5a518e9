# SwAV 1x1 forward routing: gemm8 grids under 128 tiles on conv.hip (in-tree) vs 0 (all gemm8),
# 512, everything with C % 64 == 0 on conv.hip (ab/_C_ft*.so, -DDL_FEW_TILE_1X1)
set -e
mkdir -p gpurun_out
for v in ft0 ft512 ft1000000; do
  timeout -k 10 1000 python bench/ab_native.py --lib ab/_C_$v.so --rounds 3 --timeout 280 -- python bench/swav_step.py --graph --iters 30 > gpurun_out/ft_$v.jsonl 2>&1 || { tail -20 gpurun_out/ft_$v.jsonl; exit 1; }
  echo $v; python3 scripts/ab_summary.py gpurun_out/ft_$v.jsonl
done
