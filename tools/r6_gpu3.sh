#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_native_rnn_gpu.py > gpurun_out/r6_native_rnn_gpu.log 2>&1; rc=$?
tail -25 gpurun_out/r6_native_rnn_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
PMC=1 bash tools/r6_fa_prof.sh
