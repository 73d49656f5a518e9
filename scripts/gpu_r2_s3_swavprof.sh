#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/s3_swav -o swav --output-format csv -- python bench/swav_step.py --batch 64 --iters 12 > gpurun_out/s3_swav.log 2>&1
rc=$?; echo rc=$rc; grep '^{' gpurun_out/s3_swav.log | cut -c1-200
[ $rc -ne 0 ] && exit $rc
python scripts/trace_tail_stats.py gpurun_out/s3_swav/swav_kernel_trace.csv gpurun_out/s3_swav/swav_steady_stats.csv --window 0.25 --skip_tail 0.0
rm -f gpurun_out/s3_swav/*kernel_trace.csv
python - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/s3_swav/swav_steady_stats.csv')))
ts=sum(float(r['TotalDurationNs']) for r in rows)
print("window kernel time %.1f ms" % (ts/1e6))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:30]:
    print("%6.2f%% %5d %8.1fus %s" % (float(r['TotalDurationNs'])/ts*100, int(r['Calls']), float(r['AverageNs'])/1e3, r['Name'][:90]))
PY
