#!/bin/bash
# kernel-trace stats of the ResNet-50 step replayed from a HIP graph
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/rn50g_prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/rn50g_prof -o run -- python3 -u $R/benchmarks/resnet50.py --batch 256 --steps 10 --warmup 3 --graph > $R/gpurun_out/rn50g_prof/out.log 2>&1
rc=$?
tail -3 $R/gpurun_out/rn50g_prof/out.log
f=$(find $R/gpurun_out/rn50g_prof -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && head -25 "$f" | cut -c1-220
find $R/gpurun_out/rn50g_prof -name "*kernel_trace.csv" -delete
exit $rc
