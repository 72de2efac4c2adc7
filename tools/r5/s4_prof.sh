set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash tools/llama_prof.sh && \
bash $S "step ldprobe 300 env PROBE_SHAPES=qkv,o,gate_up,down python -u benchmarks/gemm_ld_probe.py"
