set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "split_bwd" > gpurun_out/r6_fa_split_tests.log 2>&1 || { echo TESTS_FAILED; tail -50 gpurun_out/r6_fa_split_tests.log; exit 1; }
tail -3 gpurun_out/r6_fa_split_tests.log
timeout -k 10 180 python -u benchmarks/fa_bwd_split_ab.py > gpurun_out/r6_fa_split_ab.log 2>&1; rc=$?; cat gpurun_out/r6_fa_split_ab.log | tail -8; exit $rc
