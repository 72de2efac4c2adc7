#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/r6_srl_places.py > gpurun_out/r6_srl_places.log 2>&1; tail -6 gpurun_out/r6_srl_places.log
