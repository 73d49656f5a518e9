#!/bin/bash
# per-kernel stats of the eager SwAV iteration, HEAD library vs in-tree (BN-backward epilogue ring)
repo=$(cd "$(dirname "$0")/.." && pwd)
cd /tmp && export TMPDIR=/tmp
DEDLOC_NATIVE_LIB=$repo/ab/_C_base.so timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $repo/gpurun_out/kst_base -o s -- python3 $repo/bench/swav_step.py --iters 3 --warmup 2 > $repo/gpurun_out/kst_base.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $repo/gpurun_out/kst_new -o s -- python3 $repo/bench/swav_step.py --iters 3 --warmup 2 > $repo/gpurun_out/kst_new.log 2>&1 || exit $?
echo done
