# attention 2-stage ring (in-tree) vs 4-stage (ab/_C_base.so): numerics, then the B=512 micro-step
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" > gpurun_out/nb2_t.log 2>&1 || { tail -30 gpurun_out/nb2_t.log; exit 1; }
tail -1 gpurun_out/nb2_t.log
timeout -k 10 900 python bench/ab_native.py --lib ab/_C_base.so --rounds 3 --timeout 280 -- python bench/model_step.py --batch 512 --iters 6 --warmup 2 > gpurun_out/nb2_step_ab.jsonl 2>&1 || { tail -20 gpurun_out/nb2_step_ab.jsonl; exit 1; }
cat gpurun_out/nb2_step_ab.jsonl
