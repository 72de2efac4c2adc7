set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step graphtest 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_hip_graph_gpu.py tests/test_optimizer_ops_gpu.py" \
 "step rn50_graph 300 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5 --graph"
