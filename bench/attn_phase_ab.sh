# phase-offset probe: odd wave-slot blocks of the first generation sleep 2/3/4 x 1024 cycles
# (25: every odd-slot block sleeps 3072) — do co-resident blocks run in lock-step?
set -e
mkdir -p gpurun_out
for r in 1 2 3; do
for v in 2 22 23 24 25; do
  echo "nb=$v $(DEDLOC_ATTN_NBUF=$v timeout -k 10 120 python bench/attn_bench.py --batch 512 --heads 16 --seq 512 --iters 20)" | cut -c1-110 | tee -a gpurun_out/attn_phase_ab.jsonl
done
done
