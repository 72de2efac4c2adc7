#!/bin/bash
# ResNet-50 bf16 NHWC: bench (20/5) then a rocprofv3 kernel-trace profile of 5 steps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
timeout -k 10 300 python3 $R/benchmarks/resnet50.py --steps 20 --warmup 5 > $R/gpurun_out/rn50_bench.log 2>&1 || { tail -20 $R/gpurun_out/rn50_bench.log; exit 1; }
tail -2 $R/gpurun_out/rn50_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rn -o run -- python3 $R/benchmarks/resnet50.py --steps 5 --warmup 2 > $R/gpurun_out/rn50_prof.log 2>&1 || { tail -20 $R/gpurun_out/rn50_prof.log; exit 1; }
f=$(find $R/gpurun_out/prof_rn -name "*kernel_stats.csv" | head -1)
python3 $R/tools/prof_summary.py "$f" "ResNet-50 bf16 NHWC bs256" 7 > $R/gpurun_out/rn50_prof.md
head -30 $R/gpurun_out/rn50_prof.md
