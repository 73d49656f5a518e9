# SwAV concurrent passes per resolution group (--splits a,b), interleaved runs of one library
set -e
mkdir -p gpurun_out
for r in 1 2 3; do
  for sp in 1,1 1,2 2,1 2,2 1,3; do
    timeout -k 10 280 python bench/swav_step.py --graph --iters 30 --splits $sp > gpurun_out/spl_$sp.$r.log 2>&1 || { tail -20 gpurun_out/spl_$sp.$r.log; exit 1; }
    echo "splits $sp round $r $(grep -o '"value": [0-9.]*' gpurun_out/spl_$sp.$r.log)"
  done
done
