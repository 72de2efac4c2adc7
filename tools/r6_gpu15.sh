#!/bin/bash
# ops_more device kernels and the native-engine GPU suites
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_native_more_gpu.py tests/test_native_engine_gpu.py tests/test_native_engine_control_gpu.py tests/test_native_engine_book_gpu.py tests/test_native_rnn_gpu.py > gpurun_out/r6_native_gpu15.log 2>&1; tail -8 gpurun_out/r6_native_gpu15.log
