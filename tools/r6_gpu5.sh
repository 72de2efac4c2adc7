#!/bin/bash
# SRL lr debug, steady-state LLaMA-7B strict-native census, 1-GPU headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/r6_srl_debug.py > gpurun_out/r6_srl_debug.log 2>&1; tail -12 gpurun_out/r6_srl_debug.log
timeout -k 10 500 python -u tools/r6_llama_census.py llama-7b 2 > gpurun_out/r6_census.log 2>&1; rc=$?; tail -5 gpurun_out/r6_census.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6_bench2.log 2>&1 || { tail -30 gpurun_out/r6_bench2.log; exit 1; }
tail -3 gpurun_out/r6_bench2.log
