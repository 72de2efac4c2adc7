#!/bin/bash
# SRL after the output-LoD reset, native-engine GPU suites, bench with the two-wave dW
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/r6_srl_places.py > gpurun_out/r6_srl_places2.log 2>&1; tail -5 gpurun_out/r6_srl_places2.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_native_rnn_gpu.py tests/test_native_engine_control_gpu.py tests/test_native_engine_book_gpu.py tests/test_native_engine_gpu.py tests/test_native_gpu.py > gpurun_out/r6_native_suites_gpu.log 2>&1; tail -4 gpurun_out/r6_native_suites_gpu.log
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r6_bench12.log 2>&1 || { tail -20 gpurun_out/r6_bench12.log; exit 1; }
tail -2 gpurun_out/r6_bench12.log
