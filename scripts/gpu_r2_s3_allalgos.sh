#!/bin/bash
# every hipBLASLt solution vs the heuristic top-64 on the B=512 ALBERT shapes
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  timeout -k 10 280 ./bench/hip/probe_lt_allalgos "$@" > gpurun_out/allalgos_$tag.log 2>&1
  local rc=$?; echo "rc=$rc $tag"; grep -E '^\{' gpurun_out/allalgos_$tag.log | cut -c1-330
  [ $rc -ne 0 ] && { tail -5 gpurun_out/allalgos_$tag.log; exit $rc; }
  return 0
}
run wgrad_qkv wgrad 3072 1024 262144 4
run wgrad_ffn1 wgrad 4096 1024 262144 4
run wgrad_ffn2 wgrad 1024 4096 262144 4
run fwd_qkv fwd 262144 3072 1024
