#!/bin/bash
mkdir -p gpurun_out
for shape in "131072 3072 1024" "131072 1024 1024"; do
  for v in full desync1 desync2 desync4 full; do
    timeout -k 5 60 ./bench/hip/probe_$v $shape $v || exit 1
  done
done 2>&1 | tee gpurun_out/probe.log
