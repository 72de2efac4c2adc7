set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step causal 300 python -u -m pytest tests/test_causality_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider" \
 "step moe_pool 400 python -u benchmarks/train_lm.py --model ernie-moe-a3b-8l --grouped-experts --micro-batch 8 --accum 4 --steps 8 --warmup 2" \
 "step moe_fixed 400 python -u benchmarks/train_lm.py --model ernie-moe-a3b-8l --grouped-experts --micro-batch 8 --accum 4 --steps 8 --warmup 2 --fixed-batch" \
 "step bench 400 python -u bench.py --gpus 1 --steps 20 --warmup 5"
