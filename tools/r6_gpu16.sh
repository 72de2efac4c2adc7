#!/bin/bash
# ops_extra / transposed-conv device kernels plus the native suites they touch
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_native_extra_gpu.py tests/test_native_more_gpu.py tests/test_native_engine_gpu.py tests/test_native_rnn_gpu.py tests/test_native_gpu.py tests/test_native_engine_book_gpu.py > gpurun_out/r6_native_gpu16.log 2>&1; rc=$?; tail -30 gpurun_out/r6_native_gpu16.log; exit $rc
