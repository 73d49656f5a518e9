# SwAV grid sizes under concurrency: in-tree (wgrad target 256, BN apply/dx cap 2048) vs
# BN cap 512 / 768, and wgrad target 192 + BN cap 1024 (ab/_C_*.so measurement builds)
set -e
mkdir -p gpurun_out
for v in bn512 bn768 combo; do
  timeout -k 10 1000 python bench/ab_native.py --lib ab/_C_$v.so --rounds 3 --timeout 280 -- python bench/swav_step.py --graph --iters 30 > gpurun_out/gc_$v.jsonl 2>&1 || { tail -20 gpurun_out/gc_$v.jsonl; exit 1; }
  echo $v; python3 scripts/ab_summary.py gpurun_out/gc_$v.jsonl
done
