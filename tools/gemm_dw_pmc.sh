#!/bin/bash
# rocprofv3 PMC passes over benchmarks/gemm_dw_probe.py (fwd K-major, dW K-major on
# copies, dW MN-major): MFMA busy vs wave cycles, LDS traffic / conflicts, wait classes.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
A="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16"
B="GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_SALU"
C="GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_WAVES"
for pass in A B C; do
  eval cs=\$$pass
  out=/tmp/dwpmc_$pass
  timeout -s KILL 120 rocprofv3 --pmc $cs -d $out -o run -- python3 $R/benchmarks/gemm_dw_probe.py > $R/gpurun_out/dw_pmc_$pass.log 2>&1 || { echo "pass $pass failed"; tail -5 $R/gpurun_out/dw_pmc_$pass.log; exit 1; }
  db=$(find $out -name "*_results.db" | head -1)
  python3 $R/tools/rocpd_pmc.py $db gemm > $R/gpurun_out/dw_pmc_$pass.txt || exit 1
done
echo all-passes-ok
