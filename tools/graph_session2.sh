set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step rn50_graph 300 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5 --graph" \
 "step rn50_graph_global 300 env PA_CAPTURE_MODE=global python -u benchmarks/resnet50.py --batch 64 --steps 5 --warmup 2 --graph"
