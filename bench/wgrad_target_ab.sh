# conv wgrad split target: 256 workgroups (in-tree) vs 128 / 192 / 512 / 1024 (ab/_C_wg*.so, -DDL_CONV_WGRAD_TARGET)
set -e
mkdir -p gpurun_out
for v in wg128 wg192; do
  timeout -k 10 1000 python bench/ab_native.py --lib ab/_C_$v.so --rounds 3 --timeout 280 -- python bench/swav_step.py --graph --iters 30 > gpurun_out/wt_$v.jsonl 2>&1 || { tail -20 gpurun_out/wt_$v.jsonl; exit 1; }
  echo $v; python3 scripts/ab_summary.py gpurun_out/wt_$v.jsonl
done
