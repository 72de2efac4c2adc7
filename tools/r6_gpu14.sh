#!/bin/bash
# native RNN GPU tests alone and after the graph-capture tests in one process; the
# new ops_more device kernels; the SRL places check
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_native_rnn_gpu.py > gpurun_out/r6_rnn_alone.log 2>&1; tail -3 gpurun_out/r6_rnn_alone.log
timeout -k 10 500 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_hip_graph_gpu.py tests/test_inference_gpu.py tests/test_native_gpu.py tests/test_native_rnn_gpu.py > gpurun_out/r6_rnn_after_graph.log 2>&1; tail -5 gpurun_out/r6_rnn_after_graph.log
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_native_more_gpu.py > gpurun_out/r6_more_gpu.log 2>&1; tail -5 gpurun_out/r6_more_gpu.log
