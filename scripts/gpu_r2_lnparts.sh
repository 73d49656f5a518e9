#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
for T in 32768 131072; do
for P in 64 128 256 512 1024; do
T=$T DEDLOC_LN_PARTS=$P timeout -k 10 120 python -u bench/ew_bench.py > gpurun_out/lnp_${T}_$P.log 2>&1 || exit 1
echo "T=$T parts=$P $(grep ln_bwd gpurun_out/lnp_${T}_$P.log | cut -c1-120)"
done
done
