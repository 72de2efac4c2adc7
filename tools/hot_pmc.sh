#!/bin/bash
# PMC passes over the hot kernels (benchmarks/hot_kernels_only.py): one rocprofv3
# --pmc run per counter group, never combined with tracing.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
B="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR TCC_HIT_sum TCC_MISS_sum"
C="SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE GRBM_COUNT TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
for pass in A B C; do
  eval cs=\$$pass
  out=/tmp/hotpmc_$pass
  timeout -s KILL 150 rocprofv3 --pmc $cs -d $out -o run -- python3 $R/benchmarks/hot_kernels_only.py 2 > $R/gpurun_out/hot_pmc_$pass.log 2>&1 || { echo "pass $pass failed"; tail -5 $R/gpurun_out/hot_pmc_$pass.log; exit 1; }
  db=$(find $out -name "*_results.db" | head -1)
  python3 $R/tools/rocpd_pmc.py $db pa > $R/gpurun_out/hot_pmc_$pass.txt || exit 1
done
echo all-passes-ok
