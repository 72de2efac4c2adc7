#!/bin/bash
# PMC passes over the one-wave vs two-wave dW GEMM (benchmarks/gemm_dw1w_probe.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
A="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM"
B="GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM"
for pass in A B; do
  eval cs=\$$pass
  out=/tmp/dw1wpmc_$pass
  timeout -s KILL 120 rocprofv3 --pmc $cs -d $out -o run -- python3 $R/benchmarks/gemm_dw1w_probe.py > $R/gpurun_out/dw1w_pmc_$pass.log 2>&1 || { echo "pass $pass failed"; tail -5 $R/gpurun_out/dw1w_pmc_$pass.log; exit 1; }
  db=$(find $out -name "*_results.db" | head -1)
  python3 $R/tools/rocpd_pmc.py $db gemm > $R/gpurun_out/dw1w_pmc_$pass.txt || exit 1
  cat $R/gpurun_out/dw1w_pmc_$pass.txt
done
