# conv.hip forward / dgrad: workgroup target (tiles per persistent workgroup = tiles / target)
set -e
mkdir -p gpurun_out
for t in 2048 4096 1000000 1024; do
  DEDLOC_CONV_WG_TARGET=$t timeout -k 10 300 python -u bench/conv_bench.py --no_miopen --iters 20 > gpurun_out/tpw_$t.jsonl 2>&1 || { tail -20 gpurun_out/tpw_$t.jsonl; exit 1; }
done
