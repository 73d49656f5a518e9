# round-5 session A: GELU-derivative epilogues (gemm8 EPI 6/7) + attention forward variants
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "gelu or gemm" > gpurun_out/a_gemm_tests.log 2>&1
tail -1 gpurun_out/a_gemm_tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_albert_model.py tests/test_sync_free_gpu.py > gpurun_out/a_model_tests.log 2>&1
tail -1 gpurun_out/a_model_tests.log
T=262144 KINDS=fwd,fwd_gelu,fwd_gelu_d,dgrad,dgrad_dgelu,dgrad_dmul timeout -k 10 300 python bench/gemm_bench.py > gpurun_out/a_gemm_bench.jsonl 2>&1
cat gpurun_out/a_gemm_bench.jsonl
for p in 0 2 3; do
  DEDLOC_ATTN_FWD_PIPE=$p timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k attention > gpurun_out/a_attn_t$p.log 2>&1
  tail -1 gpurun_out/a_attn_t$p.log
  echo "pipe=$p" >> gpurun_out/a_attn.jsonl
  DEDLOC_ATTN_FWD_PIPE=$p timeout -k 10 120 python bench/attn_bench.py --batch 512 --heads 16 --seq 512 --iters 20 >> gpurun_out/a_attn.jsonl
done
cat gpurun_out/a_attn.jsonl
timeout -k 10 400 python bench.py --steps 5 --warmup 1 > gpurun_out/a_bench.log 2>&1
tail -1 gpurun_out/a_bench.log
