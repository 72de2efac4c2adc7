#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for mode in 0 1 2; do
  PA_ADAMW_MODE=$mode timeout -k 10 120 python -u benchmarks/adamw_bw.py >> gpurun_out/r6_adamw.log 2>&1 || { tail -20 gpurun_out/r6_adamw.log; exit 1; }
done
cat gpurun_out/r6_adamw.log
