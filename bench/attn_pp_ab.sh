# ping-pong forward: 30 = groups w >> 2, 31 = groups w & 1, 32 = w >> 2 with waves 4-7 at priority 1
set -e
mkdir -p gpurun_out
DEDLOC_ATTN_NBUF=31 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k attention > gpurun_out/attn_pp_t.log 2>&1 || { tail -30 gpurun_out/attn_pp_t.log; exit 1; }
tail -1 gpurun_out/attn_pp_t.log
for r in 1 2; do
for v in 4 30 31; do
  echo "nb=$v $(DEDLOC_ATTN_NBUF=$v timeout -k 10 120 python bench/attn_bench.py --batch 512 --heads 16 --seq 512 --iters 20)" | cut -c1-110 | tee -a gpurun_out/attn_pp_ab3.jsonl
done
done
