# BN statistics kernels' grid cap per group: 1024 (in-tree) vs 256 / 512 / 2048 (ab/_C_st*.so)
set -e
mkdir -p gpurun_out
for v in st256 st512 st2048; do
  timeout -k 10 1000 python bench/ab_native.py --lib ab/_C_$v.so --rounds 3 --timeout 280 -- python bench/swav_step.py --graph --iters 30 > gpurun_out/sc_$v.jsonl 2>&1 || { tail -20 gpurun_out/sc_$v.jsonl; exit 1; }
  echo $v; python3 scripts/ab_summary.py gpurun_out/sc_$v.jsonl
done
