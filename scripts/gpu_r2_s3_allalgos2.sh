#!/bin/bash
# random operands: forward QKV with and without the bias epilogue, every solution vs heuristic top-64
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  timeout -k 10 280 ./bench/hip/probe_lt_allalgos "$@" > gpurun_out/allalgos2_$tag.log 2>&1
  local rc=$?; echo "rc=$rc $tag"; grep -E '^\{' gpurun_out/allalgos2_$tag.log | head -4 | cut -c1-300
  [ $rc -ne 0 ] && { tail -5 gpurun_out/allalgos2_$tag.log; exit $rc; }
  return 0
}
run fwd_qkv fwd 262144 3072 1024
run fwdb_qkv fwdb 262144 3072 1024
run fwd_ffn1 fwd 262144 4096 1024
run fwd_ffn2 fwd 262144 1024 4096
