#!/bin/bash
# one-wave dW GEMM: numerics, A/B against the two-wave kernel, then the LLaMA-7B bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/r6_gemm_tests.log 2>&1 || { tail -30 gpurun_out/r6_gemm_tests.log; exit 1; }
tail -3 gpurun_out/r6_gemm_tests.log
timeout -k 10 300 python -u benchmarks/gemm_dw1w_ab.py > gpurun_out/r6_dw1w_ab.jsonl 2>&1 || { tail -20 gpurun_out/r6_dw1w_ab.jsonl; exit 1; }
cat gpurun_out/r6_dw1w_ab.jsonl
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r6_bench8.log 2>&1 || { tail -20 gpurun_out/r6_bench8.log; exit 1; }
tail -2 gpurun_out/r6_bench8.log
