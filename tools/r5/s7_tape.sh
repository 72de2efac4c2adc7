set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step tape_gpu 600 python -u -m pytest tests/test_no_torch_autograd_gpu.py tests/test_rccl_comm_gpu.py tests/test_fused_epilogue_gpu.py tests/test_causality_gpu.py -v --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "step models 600 python -u -m pytest tests/test_models_gpu.py tests/test_tape_gpu.py tests/test_hybrid_gpu.py tests/test_sharding_overlap_gpu.py tests/test_overlap_update_gpu.py -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "step bench 400 python -u bench.py --gpus 1 --steps 20 --warmup 5"
