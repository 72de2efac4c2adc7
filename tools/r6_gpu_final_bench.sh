#!/bin/bash
# round-end rehearsal, part 2: smoke() then the 1-GPU headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_final_smoke.log 2>&1 || { tail -20 gpurun_out/r6_final_smoke.log; exit 1; }
tail -2 gpurun_out/r6_final_smoke.log
timeout -k 10 700 python -u bench.py > gpurun_out/r6_final_bench.log 2>&1
rc=$?
tail -5 gpurun_out/r6_final_bench.log
exit $rc
