# SwAV gemm8 weight-gradient split target: 256 CUs (in-tree) vs 128 / 192 (ab/_C_wc*.so, -DDL_WGRAD_CUS)
set -e
mkdir -p gpurun_out
for v in wc128 wc192; do
  timeout -k 10 1000 python bench/ab_native.py --lib ab/_C_$v.so --rounds 3 --timeout 280 -- python bench/swav_step.py --graph --iters 30 > gpurun_out/wc_$v.jsonl 2>&1 || { tail -20 gpurun_out/wc_$v.jsonl; exit 1; }
  echo $v; python3 scripts/ab_summary.py gpurun_out/wc_$v.jsonl
done
