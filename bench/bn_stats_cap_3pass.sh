# BN statistics grid cap re-checked with three concurrent passes: 256 (in-tree) vs 128 / 512
set -e
mkdir -p gpurun_out
for v in st128 st512; do
  timeout -k 10 1000 python bench/ab_native.py --lib ab/_C_$v.so --rounds 3 --timeout 280 -- python bench/swav_step.py --graph --iters 30 > gpurun_out/s3_$v.jsonl 2>&1 || { tail -20 gpurun_out/s3_$v.jsonl; exit 1; }
  echo $v; python3 scripts/ab_summary.py gpurun_out/s3_$v.jsonl
done
