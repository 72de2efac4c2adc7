#!/bin/bash
# SRL per-place losses, native recurrent on the GPU, one-wave dW GEMM numerics + A/B, bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/r6_srl_places.py > gpurun_out/r6_srl_places.log 2>&1; tail -6 gpurun_out/r6_srl_places.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_native_rnn_gpu.py -k "layout_ops" > gpurun_out/r6_native_layout_gpu2.log 2>&1; tail -4 gpurun_out/r6_native_layout_gpu2.log
bash tools/r6_gpu8.sh
