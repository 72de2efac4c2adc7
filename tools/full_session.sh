set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step suite 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "step bench 400 python -u bench.py --gpus 1 --steps 20 --warmup 5" \
 "step rn50 300 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5"
