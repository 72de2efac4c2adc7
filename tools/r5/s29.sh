set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step t29 500 python -u -m pytest tests/test_conv_gpu.py tests/test_convnd_gpu.py tests/test_bf16_state_gpu.py tests/test_dygraph_gpu.py tests/test_eager_engine_gpu.py tests/test_hip_graph_gpu.py -q --timeout 200 --timeout-method thread -p no:cacheprovider" \
 "step bnab29 300 python -u benchmarks/bn_apply_ab.py" \
 "step rnA1 300 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step rnB1 300 env PA_BN_APPLY=0 PA_BN_EW_CAP=2048 PA_BN_DX=0 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step rnA2 300 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step rnB2 300 env PA_BN_APPLY=0 PA_BN_EW_CAP=2048 PA_BN_DX=0 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5"
