# round-5 session B: multi-peer collaboration on one GPU (peers share the device -> gloo data plane),
# one micro-step per peer per global step (the 8-GPU headline's shape), after the protocol changes
set -e
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --gpus 2 --allow_shared_device --micro_batch 256 --target_batch_size 512 --steps 6 --warmup 2 > gpurun_out/b_2peers.log 2>&1
tail -1 gpurun_out/b_2peers.log
timeout -k 10 400 python bench.py --gpus 4 --allow_shared_device --micro_batch 128 --target_batch_size 512 --steps 6 --warmup 2 > gpurun_out/b_4peers.log 2>&1
tail -1 gpurun_out/b_4peers.log
timeout -k 10 300 python bench.py --gpus 1 --micro_batch 512 --target_batch_size 512 --steps 6 --warmup 2 > gpurun_out/b_1peer.log 2>&1
tail -1 gpurun_out/b_1peer.log
