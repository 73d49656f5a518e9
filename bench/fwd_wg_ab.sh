# conv forward workgroup target 1024 (in-tree) vs 512 / 2048 (ab/_C_fw*.so); BN stats cap 256 repeat
set -e
mkdir -p gpurun_out
for v in fw512 fw2048; do
  timeout -k 10 1000 python bench/ab_native.py --lib ab/_C_$v.so --rounds 3 --timeout 280 -- python bench/swav_step.py --graph --iters 30 > gpurun_out/fw_$v.jsonl 2>&1 || { tail -20 gpurun_out/fw_$v.jsonl; exit 1; }
  echo $v; python3 scripts/ab_summary.py gpurun_out/fw_$v.jsonl
done
timeout -k 10 1200 python bench/ab_native.py --lib ab/_C_st256.so --rounds 4 --timeout 280 -- python bench/swav_step.py --graph --iters 30 > gpurun_out/fw_st256.jsonl 2>&1 || { tail -20 gpurun_out/fw_st256.jsonl; exit 1; }
echo st256; python3 scripts/ab_summary.py gpurun_out/fw_st256.jsonl
