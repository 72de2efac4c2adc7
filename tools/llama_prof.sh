#!/bin/bash
# rocprofv3 kernel trace of the LLaMA-7B bench step (3 steps incl. 1 warmup)
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_llama -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/llama_prof.log 2>&1 || { tail -20 $R/gpurun_out/llama_prof.log; exit 1; }
tail -2 $R/gpurun_out/llama_prof.log
