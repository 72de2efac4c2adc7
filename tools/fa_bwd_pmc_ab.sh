#!/bin/bash
# PMC passes over the flash-attention backward kernel variants named in $1
# (e.g. "4 5"): MFMA busy vs cycles, LDS traffic / conflicts, wait classes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
A="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16"
B="GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_SALU"
for v in $1; do
  for pass in A B; do
    eval cs=\$$pass
    out=/tmp/fabpmc_${v}_${pass}
    timeout -s KILL 90 rocprofv3 --pmc $cs -d $out -o run -- python3 $R/benchmarks/fa_bwd_only.py $v 3 > $R/gpurun_out/fab_pmc_${v}_${pass}.log 2>&1 || { echo "pass $v $pass failed"; tail -3 $R/gpurun_out/fab_pmc_${v}_${pass}.log; exit 1; }
    db=$(find $out -name "*_results.db" | head -1)
    python3 $R/tools/rocpd_pmc.py $db fa_bwd_kernel > $R/gpurun_out/fab_pmc_${v}_${pass}.txt || exit 1
  done
done
echo all-passes-ok
