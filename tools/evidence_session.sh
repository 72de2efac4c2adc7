set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step eager_probe 300 env FLAGS_count_aten=1 python -u tools/eager_trace_probe.py" \
 "step rn50_graph 300 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5 --graph" \
 "step rn50 300 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5"
