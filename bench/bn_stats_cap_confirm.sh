# BN statistics grid cap: adopted 256 (in-tree) vs previous 1024 and vs 128 (ab/_C_st*.so)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_swav_kernels_gpu.py tests/test_swav.py > gpurun_out/scc_t.log 2>&1 || { tail -40 gpurun_out/scc_t.log; exit 1; }
tail -1 gpurun_out/scc_t.log
for v in st1024 st128; do
  timeout -k 10 1200 python bench/ab_native.py --lib ab/_C_$v.so --rounds 4 --timeout 280 -- python bench/swav_step.py --graph --iters 30 > gpurun_out/scc_$v.jsonl 2>&1 || { tail -20 gpurun_out/scc_$v.jsonl; exit 1; }
  echo $v; python3 scripts/ab_summary.py gpurun_out/scc_$v.jsonl
done
