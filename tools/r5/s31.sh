set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step t31 500 python -u -m pytest tests/test_conv_gpu.py tests/test_convnd_gpu.py tests/test_bf16_state_gpu.py tests/test_dygraph_gpu.py tests/test_eager_engine_gpu.py tests/test_hip_graph_gpu.py tests/test_native_engine_gpu.py -q --timeout 200 --timeout-method thread -p no:cacheprovider" \
 "step rnA1 300 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step rnB1 300 env PA_BN_APPLY=0 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step rnA2 300 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step rnB2 300 env PA_BN_APPLY=0 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5"
