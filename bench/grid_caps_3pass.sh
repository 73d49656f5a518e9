# grid caps re-checked with three concurrent passes (splits (2,1)): in-tree (BN apply 768, wgrad 192)
# vs BN apply 512 / 1024 and wgrad 128 / 256 (ab/_C_*.so)
set -e
mkdir -p gpurun_out
for v in ap512 ap1024 wg128 wg256; do
  timeout -k 10 1000 python bench/ab_native.py --lib ab/_C_$v.so --rounds 3 --timeout 280 -- python bench/swav_step.py --graph --iters 30 > gpurun_out/g3_$v.jsonl 2>&1 || { tail -20 gpurun_out/g3_$v.jsonl; exit 1; }
  echo $v; python3 scripts/ab_summary.py gpurun_out/g3_$v.jsonl
done
