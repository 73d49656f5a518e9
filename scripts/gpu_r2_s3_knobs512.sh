#!/bin/bash
# LayerNorm-backward grid and weight-gradient token splits at micro-batch 512 (interleaved, one box)
mkdir -p gpurun_out
export PYTHONPATH=$PWD
for r in 1 2; do
  for v in default lnparts1024 lnparts256 wgs2 wgs8; do
    case $v in
      default) env="";;
      lnparts1024) env="DEDLOC_LN_PARTS=1024";;
      lnparts256) env="DEDLOC_LN_PARTS=256";;
      wgs2) env="DEDLOC_WGRAD_SPLITS=2";;
      wgs8) env="DEDLOC_WGRAD_SPLITS=8";;
    esac
    env $env timeout -k 10 240 python -u bench/model_step.py --impl dedloc --batch 512 --iters 6 --warmup 2 > gpurun_out/knob_${v}_$r.log 2>&1 || { echo "fail $v"; tail -5 gpurun_out/knob_${v}_$r.log; exit 1; }
    echo "$v $r $(grep '^{' gpurun_out/knob_${v}_$r.log | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["samples_per_s"],1))')"
  done
done
