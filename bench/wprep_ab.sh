# SwAV data-gradient weight preparation: own stream (default, 1) vs the main stream (0), three passes
set -e
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in 1 0; do
    timeout -k 10 280 python bench/swav_step.py --graph --iters 30 --model_attr dgrad_weights_stream=$v > gpurun_out/wp_$v.$r.log 2>&1 || { tail -20 gpurun_out/wp_$v.$r.log; exit 1; }
    echo "dgrad_weights_stream $v round $r $(grep -o '"value": [0-9.]*' gpurun_out/wp_$v.$r.log)"
  done
done
