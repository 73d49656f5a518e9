# conv data gradient: parity-class grids merged into one launch (MULTI kernel, per-job tpw, jobs
# interleaved over the XCDs) vs HEAD (ab/_C_base.so); conv_bench sweeps the merge threshold
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv.py tests/test_swav_kernels_gpu.py tests/test_swav.py tests/test_swav_parity_gpu.py > gpurun_out/dm3_t.log 2>&1 || { tail -40 gpurun_out/dm3_t.log; exit 1; }
tail -1 gpurun_out/dm3_t.log
for th in 0 512 100000; do
  DEDLOC_CONV_MERGE_TILES=$th timeout -k 10 300 python -u bench/conv_bench.py --no_miopen --iters 20 > gpurun_out/dm3_conv_shapes_$th.jsonl 2>&1 || { tail -20 gpurun_out/dm3_conv_shapes_$th.jsonl; exit 1; }
done
timeout -k 10 900 python bench/ab_native.py --lib ab/_C_base.so --rounds 3 --timeout 280 -- python bench/swav_step.py --graph --iters 30 > gpurun_out/dm3_swav_ab.jsonl 2>&1 || { tail -20 gpurun_out/dm3_swav_ab.jsonl; exit 1; }
python3 scripts/ab_summary.py gpurun_out/dm3_swav_ab.jsonl
