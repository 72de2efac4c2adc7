#!/bin/bash
# rocprofv3 kernel trace of the flash-attention backward A/B (split vs fused) + PMC of the split kernels
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_fa -o run -- python3 $R/benchmarks/fa_bwd_split_ab.py > $R/gpurun_out/fa_prof.log 2>&1 || { tail -20 $R/gpurun_out/fa_prof.log; exit 1; }
db=$(find $R/gpurun_out/prof_fa -name "*_results.db" | head -1)
python3 $R/tools/rocpd_summary.py $db "FA bwd A/B" > $R/gpurun_out/fa_prof_summary.md && head -30 $R/gpurun_out/fa_prof_summary.md
if [ -n "$PMC" ]; then
  for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"; do
    n=$((n+1))
    timeout -s KILL 90 rocprofv3 --pmc $pass -d /tmp/fapmc$n -o run -- python3 $R/benchmarks/fa_bwd_split_ab.py > $R/gpurun_out/fa_pmc$n.log 2>&1 || { echo "pmc pass $n failed"; exit 1; }
    db=$(find /tmp/fapmc$n -name "*_results.db" | head -1)
    python3 $R/tools/rocpd_pmc.py $db fab:: > $R/gpurun_out/fa_pmc$n.txt || exit 1
    cat $R/gpurun_out/fa_pmc$n.txt
  done
fi
