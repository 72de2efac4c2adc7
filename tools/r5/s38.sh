#!/bin/bash
# LLaMA-7B bench step under rocprofv3 kernel trace after the transpose128 change
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_llama38 -o run -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof_llama38.log 2>&1
