#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/r6_srl_debug.py > gpurun_out/r6_srl_debug.log 2>&1; cat gpurun_out/r6_srl_debug.log | tail -15
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "split_bwd" > gpurun_out/r6_fa_split_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6_fa_split_tests.log; exit 1; }
tail -2 gpurun_out/r6_fa_split_tests.log
timeout -k 10 180 python -u benchmarks/fa_bwd_split_ab.py > gpurun_out/r6_fa_split_ab.log 2>&1; rc=$?; tail -8 gpurun_out/r6_fa_split_ab.log; exit $rc
