#!/bin/bash
# round-end rehearsal, part 1: the whole GPU test suite in one process
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1050 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r6_final_gpu_suite.log 2>&1
rc=$?
tail -25 gpurun_out/r6_final_gpu_suite.log
exit $rc
