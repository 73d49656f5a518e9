#!/bin/bash
# exhaustive hipBLASLt autotune at micro-batch 512 -> tuning database; then the same step from the
# database, the heuristic-only autotune (A/B on one box) and the headline bench
mkdir -p gpurun_out
export PYTHONPATH=$PWD
rm -f gpurun_out/lt_tuning_gfx950.txt
step() {
  local log=$1; shift
  timeout -k 10 "$@" > "$log" 2>&1
  local rc=$?
  echo "rc=$rc $*"; grep -E '^\{|\[lt\] plan' "$log" | tail -24 | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; tail -30 "$log"; exit $rc; fi
}
DEDLOC_LT_DB=/nonexistent DEDLOC_LT_DB_OUT=gpurun_out/lt_tuning_gfx950.txt step gpurun_out/ltdb_tune.log 500 python -u bench/model_step.py --impl dedloc --batch 512 --iters 6 --warmup 2
wc -l gpurun_out/lt_tuning_gfx950.txt
DEDLOC_LT_DB=gpurun_out/lt_tuning_gfx950.txt DEDLOC_LT_DEBUG=1 step gpurun_out/ltdb_use.log 300 python -u bench/model_step.py --impl dedloc --batch 512 --iters 6 --warmup 2
grep -c "tuning database solution" gpurun_out/ltdb_use.log
DEDLOC_LT_DB=/nonexistent DEDLOC_LT_EXHAUSTIVE=0 step gpurun_out/ltdb_heur.log 300 python -u bench/model_step.py --impl dedloc --batch 512 --iters 6 --warmup 2
DEDLOC_LT_DB=gpurun_out/lt_tuning_gfx950.txt step gpurun_out/ltdb_bench.log 400 python -u bench.py
