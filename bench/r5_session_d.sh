# round-5 session D: lean dK/dV exponent (key-length masks) + the SwAV graph probe with the real peer
mkdir -p gpurun_out
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_kernels_fuzz_gpu.py -k "attention or attn" > gpurun_out/d_attn_tests.log 2>&1
tail -1 gpurun_out/d_attn_tests.log
for pad in 0.0 0.25; do
  timeout -k 10 120 python bench/attn_bench.py --batch 512 --heads 16 --seq 512 --iters 20 --pad $pad >> gpurun_out/d_attn.jsonl
done
cat gpurun_out/d_attn.jsonl
set +e
timeout -k 10 700 python bench/graph_selfwait_probe.py > gpurun_out/d_graph_probe.log 2>&1
echo "probe rc=$?"
grep -E '^case=|@@' gpurun_out/d_graph_probe.log
