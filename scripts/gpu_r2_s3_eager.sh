#!/bin/bash
# the measured baseline at larger micro-batches (reference stack: HF AlbertForPreTraining + torch LAMB)
mkdir -p gpurun_out
export PYTHONPATH=$PWD
for B in 128 256; do
  timeout -k 10 400 python -u bench.py --impl eager --micro_batch $B --steps 1 --warmup 1 > gpurun_out/eager_mb$B.log 2>&1
  rc=$?; echo "rc=$rc B=$B"; grep '^{' gpurun_out/eager_mb$B.log | cut -c1-250
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/eager_mb$B.log; exit $rc; fi
done
