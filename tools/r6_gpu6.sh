#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/r6_crf_debug.py > gpurun_out/r6_crf_debug.log 2>&1; tail -30 gpurun_out/r6_crf_debug.log
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_llama6 -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/llama_prof6.log 2>&1 || { tail -20 $R/gpurun_out/llama_prof6.log; exit 1; }
db=$(find $R/gpurun_out/prof_llama6 -name "*_results.db" | head -1)
python3 $R/tools/rocpd_summary.py $db "LLaMA-7B bench step (3 steps incl. warmup), round 6" > $R/gpurun_out/llama_prof6_summary.md && head -45 $R/gpurun_out/llama_prof6_summary.md
