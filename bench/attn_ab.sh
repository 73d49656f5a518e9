set -e
for p in 0 2 3 1; do
  DEDLOC_ATTN_FWD_PIPE=$p timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k attention > gpurun_out/attn_t$p.log 2>&1
  tail -1 gpurun_out/attn_t$p.log
done
for r in 1 2; do
for p in 0 2 3 1; do
  echo "pipe=$p" >> gpurun_out/attn_ab.jsonl
  DEDLOC_ATTN_FWD_PIPE=$p timeout -k 10 120 python bench/attn_bench.py --batch 512 --heads 16 --seq 512 --iters 20 >> gpurun_out/attn_ab.jsonl
done
done
cat gpurun_out/attn_ab.jsonl
