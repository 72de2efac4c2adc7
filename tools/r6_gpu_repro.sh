#!/bin/bash
# order-dependence check of test_native_sequence_ops_device_kernels, then smoke + bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_native_engine_book_gpu.py tests/test_native_engine_control_gpu.py tests/test_native_engine_gpu.py tests/test_optimizer_ops_gpu.py > gpurun_out/r6_repro.log 2>&1
rc=$?
tail -12 gpurun_out/r6_repro.log
case $rc in 124|134|137|139) exit $rc;; esac
bash tools/r6_gpu_final_bench.sh
