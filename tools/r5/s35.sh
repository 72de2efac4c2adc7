#!/bin/bash
# transpose A/B: 64x64 (round 2-4) vs 128x128 grouped / row-major, then the kernel tests
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/tr_ab.jsonl
: > $O
timeout -k 10 120 python -u -m pytest -x -q --timeout 100 --timeout-method thread tests/test_kernels_gpu.py -k transpose > gpurun_out/tr_test.log 2>&1 &&
PA_TRANSPOSE=0 timeout -k 10 120 python -u benchmarks/transpose_bench.py >> $O &&
PA_TRANSPOSE=1 PA_TR_GROUP=8 timeout -k 10 120 python -u benchmarks/transpose_bench.py >> $O &&
PA_TRANSPOSE=1 PA_TR_GROUP=0 timeout -k 10 120 python -u benchmarks/transpose_bench.py >> $O &&
PA_TRANSPOSE=1 PA_TR_GROUP=4 timeout -k 10 120 python -u benchmarks/transpose_bench.py >> $O &&
PA_TRANSPOSE=1 PA_TR_GROUP=16 timeout -k 10 120 python -u benchmarks/transpose_bench.py >> $O
