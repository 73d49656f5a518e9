#!/bin/bash
# wide-row LayerNorm backward (D = 2048 / 4096): numerics, then albert-xxlarge through the kernels
mkdir -p gpurun_out
export PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_kernels_fuzz_gpu.py -q -k "layernorm" --timeout 300 --timeout-method thread -p no:warnings > gpurun_out/wideln_pytest.log 2>&1
rc=$?; grep -E "passed|failed|Falsifying|^E  " gpurun_out/wideln_pytest.log | head -20; [ $rc -ne 0 ] && exit $rc
python - <<'PY'
from dedloc_amd.models.albert import AlbertConfig
AlbertConfig(vocab_size=30000, embedding_size=128, hidden_size=4096, num_hidden_layers=12, num_hidden_groups=1,
             num_attention_heads=64, intermediate_size=16384, inner_group_num=1).save_pretrained("gpurun_out/xxlarge_cfg")
PY
timeout -k 10 400 python -u bench/model_step.py --config gpurun_out/xxlarge_cfg --batch 64 --iters 4 --warmup 2 > gpurun_out/cfg_xxlarge.log 2>&1
rc=$?; grep '^{' gpurun_out/cfg_xxlarge.log | cut -c1-220; [ $rc -ne 0 ] && tail -5 gpurun_out/cfg_xxlarge.log
exit $rc
