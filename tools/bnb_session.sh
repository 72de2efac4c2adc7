set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step tests 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_profiler_gpu.py tests/test_eager_engine_gpu.py tests/test_native_engine_book_gpu.py" \
 "step rn50 300 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step rn50_nobnb 300 env FLAGS_conv_bn_bwd_stats=0 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step rn50_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn8 -o run -- python3 benchmarks/resnet50.py --batch 256 --steps 5 --warmup 2"
