#!/bin/bash
# SwAV: exhaustive hipBLASLt search for the (small) 1x1-conv / head GEMMs vs the heuristic autotune
mkdir -p gpurun_out
export PYTHONPATH=$PWD
rm -f gpurun_out/lt_tuning_swav.txt
timeout -k 10 400 python -u bench/swav_step.py --batch 64 --iters 20 > gpurun_out/swavlt_heur_1.log 2>&1 || exit 1
grep '^{' gpurun_out/swavlt_heur_1.log | cut -c1-120
DEDLOC_LT_EXHAUSTIVE=1 DEDLOC_LT_EXHAUSTIVE_MIN_GFLOP=0.5 DEDLOC_LT_DB_OUT=gpurun_out/lt_tuning_swav.txt timeout -k 10 600 python -u bench/swav_step.py --batch 64 --iters 20 > gpurun_out/swavlt_tune.log 2>&1 || { tail -5 gpurun_out/swavlt_tune.log; exit 1; }
grep '^{' gpurun_out/swavlt_tune.log | cut -c1-120; wc -l gpurun_out/lt_tuning_swav.txt
cat dedloc_amd/lt_tuning_gfx950.txt gpurun_out/lt_tuning_swav.txt > gpurun_out/lt_tuning_both.txt
for r in 1 2; do
  timeout -k 10 400 python -u bench/swav_step.py --batch 64 --iters 20 > gpurun_out/swavlt_heur_r$r.log 2>&1 || exit 1
  echo "heur $r $(grep '^{' gpurun_out/swavlt_heur_r$r.log | cut -c1-110)"
  DEDLOC_LT_DB=gpurun_out/lt_tuning_both.txt timeout -k 10 400 python -u bench/swav_step.py --batch 64 --iters 20 > gpurun_out/swavlt_db_r$r.log 2>&1 || exit 1
  echo "db   $r $(grep '^{' gpurun_out/swavlt_db_r$r.log | cut -c1-110)"
done
