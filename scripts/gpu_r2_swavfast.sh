#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest tests/test_swav.py tests/test_conv.py -q -m gpu -x --timeout 200 --timeout-method thread > gpurun_out/swf_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/swf_pytest.log; [ $rc -ne 0 ] && tail -30 gpurun_out/swf_pytest.log && exit $rc
for i in 1 2; do
timeout -k 10 500 python -u bench/swav_step.py --batch 64 --iters 10 > gpurun_out/swf_$i.log 2>&1 || exit 1
echo "run $i $(grep '^{' gpurun_out/swf_$i.log | cut -c1-140)"
done
