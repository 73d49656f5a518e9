#!/bin/bash
# attention kernel variants at micro-batch 512 (interleaved, one box): default vs 8-wave forward vs
# two-key-sub-block dK/dV
mkdir -p gpurun_out
export PYTHONPATH=$PWD
for r in 1 2; do
  for v in default nw8 ks2; do
    case $v in
      default) env="";;
      nw8) env="DEDLOC_ATTN_NW=8";;
      ks2) env="DEDLOC_ATTN_DKDV_KS=2";;
    esac
    env $env timeout -k 10 240 python -u bench/model_step.py --impl dedloc --batch 512 --iters 6 --warmup 2 > gpurun_out/attnab_${v}_$r.log 2>&1 || { echo "fail $v"; tail -5 gpurun_out/attnab_${v}_$r.log; exit 1; }
    echo "$v $r $(grep '^{' gpurun_out/attnab_${v}_$r.log | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["samples_per_s"],1))')"
  done
done
