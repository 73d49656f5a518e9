# SwAV pass stream priorities, interleaved runs of one library: default vs the first (largest)
# pass on a high-priority stream (main_priority=-1); side passes at high priority were measured
# first (2600 vs 3340 samples/s)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_swav.py > gpurun_out/mp_t.log 2>&1 || { tail -40 gpurun_out/mp_t.log; exit 1; }
tail -1 gpurun_out/mp_t.log
for r in 1 2 3; do
  for pr in 0 -1; do
    timeout -k 10 280 python bench/swav_step.py --graph --iters 30 --model_attr main_priority=$pr > gpurun_out/mp_$pr.$r.log 2>&1 || { tail -20 gpurun_out/mp_$pr.$r.log; exit 1; }
    echo "main_priority $pr round $r $(grep -o '"value": [0-9.]*' gpurun_out/mp_$pr.$r.log)"
  done
done
