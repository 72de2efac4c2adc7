set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step gstem_dev 120 env SET_DEVICE=1 python -u tools/graph_debug.py stem" \
 "step gstep_dev 150 env SET_DEVICE=1 python -u tools/graph_debug.py step" \
 "step rn50_graph 300 env PA_SET_DEVICE=1 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5 --graph" \
 "step rn50 300 env PA_SET_DEVICE=1 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5"
