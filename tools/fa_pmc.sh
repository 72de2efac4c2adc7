#!/bin/bash
# Flash-attention PMC passes (one rocprofv3 run per counter group; never combined
# with tracing).  Writes per-pass summaries to gpurun_out/fa_pmc_*.txt.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
B="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR TCC_HIT_sum TCC_MISS_sum"
for kind in fwd bwd; do
  for pass in A B; do
    eval cs=\$$pass
    out=/tmp/fapmc_${kind}_${pass}
    args=3; [ $kind = bwd ] && args="4 3"  # bwd: default variant 4, 3 reps
    timeout -s KILL 90 rocprofv3 --pmc $cs -d $out -o run -- python3 $R/benchmarks/fa_${kind}_only.py $args > $R/gpurun_out/fa_pmc_${kind}_${pass}.log 2>&1 || { echo "pass $kind $pass failed"; exit 1; }
    db=$(find $out -name "*_results.db" | head -1)
    python3 $R/tools/rocpd_pmc.py $db fa_ > $R/gpurun_out/fa_pmc_${kind}_${pass}.txt || exit 1
  done
done
echo all-passes-ok
