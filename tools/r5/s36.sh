#!/bin/bash
# transpose128 default: kernel tests, transpose bench, LLaMA-7B bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_epilogue_gpu.py > gpurun_out/tr_test2.log 2>&1 &&
timeout -k 10 120 python -u benchmarks/transpose_bench.py > gpurun_out/tr_default.jsonl &&
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_tr.log 2>&1
