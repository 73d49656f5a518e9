#!/bin/bash
# Per-shape conv timings (ours only, then ours vs MIOpen) on the current tree.
mkdir -p gpurun_out
timeout -k 10 300 python -u bench/conv_bench.py --no_miopen --iters 20 > gpurun_out/r5_conv_shapes_ours.jsonl 2> gpurun_out/r5_conv_shapes_ours.err &&
timeout -k 10 700 python -u bench/conv_bench.py --iters 10 > gpurun_out/r5_conv_shapes_vs_miopen.jsonl 2> gpurun_out/r5_conv_shapes_vs_miopen.err
