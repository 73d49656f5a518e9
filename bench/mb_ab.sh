# ALBERT-large micro-step at B=512 vs B=1024 (bench/model_step.py), interleaved
set -e
mkdir -p gpurun_out
for r in 1 2; do
  for b in 512 1024; do
    timeout -k 10 400 python bench/model_step.py --batch $b --iters 4 --warmup 2 > gpurun_out/mb_$b.$r.log 2>&1 || { tail -20 gpurun_out/mb_$b.$r.log; exit 1; }
    echo "batch $b round $r $(grep -o '"samples_per_s": [0-9.]*' gpurun_out/mb_$b.$r.log) $(grep -o '"peak[a-z_]*": [0-9.]*' gpurun_out/mb_$b.$r.log)"
  done
done
