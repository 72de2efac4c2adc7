set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step fused 300 python -u -m pytest tests/test_fused_epilogue_gpu.py -v --timeout 200 --timeout-method thread -p no:cacheprovider" \
 "step kern 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_tape_gpu.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider" \
 "step bench 400 python -u bench.py --gpus 1 --steps 20 --warmup 5"
