# gemm8 BNBWD: BN coefficients in LDS, BN input read one pass ahead (in-tree) vs HEAD
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv.py tests/test_swav_kernels_gpu.py tests/test_swav.py tests/test_swav_parity_gpu.py > gpurun_out/bp_t.log 2>&1 || { tail -40 gpurun_out/bp_t.log; exit 1; }
tail -1 gpurun_out/bp_t.log
timeout -k 10 900 python bench/ab_native.py --lib ab/_C_base.so --rounds 3 --timeout 280 -- python bench/swav_step.py --graph --iters 30 > gpurun_out/bp_swav_ab.jsonl 2>&1 || { tail -20 gpurun_out/bp_swav_ab.jsonl; exit 1; }
python3 -c "
import json
rows=[json.loads(l) for l in open('gpurun_out/bp_swav_ab.jsonl') if l.startswith('{')]
for arm in 'AB': print(arm, [round(r['value'],1) for r in rows if r['arm']==arm])
"
