# A/B of the attention ring depth / occupancy variants (DEDLOC_ATTN_NBUF: 4 = shipped, 2 / 3 = ring
# depth at QS = 2, 12 / 13 = QS = 1 at 4 / 3 waves per SIMD)
set -e
mkdir -p gpurun_out
for v in 12 13; do
  DEDLOC_ATTN_NBUF=$v timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k attention > gpurun_out/attn_nb_t$v.log 2>&1
  echo "nb=$v $(tail -1 gpurun_out/attn_nb_t$v.log)"
done
for r in 1 2 3; do
for v in 4 2 12 13; do
  echo "nb=$v $(DEDLOC_ATTN_NBUF=$v timeout -k 10 120 python bench/attn_bench.py --batch 512 --heads 16 --seq 512 --iters 20)" | tee -a gpurun_out/attn_nb_ab2.jsonl
done
done
