#!/bin/bash
mkdir -p gpurun_out
export PYTHONPATH=$PWD
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r2_prof256 -o albert --output-format csv -- python bench/model_step.py --impl dedloc --batch 256 --iters 4 --warmup 2 > gpurun_out/r2_prof256.log 2>&1
rc=$?; echo rc=$rc; grep '^{' gpurun_out/r2_prof256.log | cut -c1-200
[ $rc -ne 0 ] && exit $rc
python scripts/trace_tail_stats.py gpurun_out/r2_prof256/albert_kernel_trace.csv gpurun_out/r2_prof256/albert_b256_steady_stats.csv --window 0.9 --skip_tail 0.0
python - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/r2_prof256/albert_kernel_trace.csv')))
ts=sorted((int(r['Start_Timestamp']),int(r['End_Timestamp'])) for r in rows)
end=ts[-1][1]; start=end-int(0.5e9)
busy=0; cur_s=cur_e=None
for s,e in ts:
    if e<start: continue
    s=max(s,start)
    if cur_e is None or s>cur_e:
        if cur_e is not None: busy+=cur_e-cur_s
        cur_s,cur_e=s,e
    else: cur_e=max(cur_e,e)
busy+=cur_e-cur_s
print("last 0.5 s: GPU busy %.1f%%" % (100*busy/(end-start)))
PY
rm -f gpurun_out/r2_prof256/*kernel_trace.csv
