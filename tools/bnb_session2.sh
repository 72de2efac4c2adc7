set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py" \
 "step rn50 300 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step rn50_nobnb 300 env FLAGS_conv_bn_bwd_stats=0 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step rn50_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn9 -o run -- python3 benchmarks/resnet50.py --batch 256 --steps 5 --warmup 2" \
 "step direct 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_direct_sharding_gpu.py"
