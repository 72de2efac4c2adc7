set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step t32 400 env PA_BN_RED_UNR=1 python -u -m pytest tests/test_conv_gpu.py tests/test_dygraph_gpu.py -q --timeout 200 --timeout-method thread -p no:cacheprovider" \
 "step rnA1 300 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step rnR1 300 env PA_BN_RED_UNR=1 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step rnD1 300 env PA_BN_DX=1 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step rnA2 300 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step rnR2 300 env PA_BN_RED_UNR=1 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step rnD2 300 env PA_BN_DX=1 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5"
