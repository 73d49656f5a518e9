#!/bin/bash
# composed attention for head_dim 128: numerics on the card, then albert-xlarge-v2 model steps
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_attention_composed.py -v --timeout 200 --timeout-method thread -p no:warnings > gpurun_out/xlarge_pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|^E  " gpurun_out/xlarge_pytest.log | head -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench/model_step.py --config albert-xlarge-v2 --batch 64 --iters 5 --warmup 2 > gpurun_out/cfg_xlarge.log 2>&1
rc=$?; grep '^{' gpurun_out/cfg_xlarge.log | cut -c1-260; [ $rc -ne 0 ] && tail -8 gpurun_out/cfg_xlarge.log
exit $rc
