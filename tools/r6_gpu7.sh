#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/r6_srl_bisect.py > gpurun_out/r6_srl_bisect.log 2>&1; tail -8 gpurun_out/r6_srl_bisect.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_native_rnn_gpu.py -k "layout_ops" > gpurun_out/r6_native_layout_gpu.log 2>&1; tail -12 gpurun_out/r6_native_layout_gpu.log
