set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step gstem 120 python -u tools/graph_debug.py stem" \
 "step gfwd 120 python -u tools/graph_debug.py fwd" \
 "step gbwd 120 python -u tools/graph_debug.py bwd" \
 "step gstep 120 python -u tools/graph_debug.py step" \
 "step gstem_fp32 120 env NO_AMP=1 python -u tools/graph_debug.py stem" \
 "step seqgpu 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_native_engine_gpu.py"
