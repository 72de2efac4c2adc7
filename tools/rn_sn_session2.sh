set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step convtests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_optimizer_ops_gpu.py tests/test_aten_native_gpu.py tests/test_eager_engine_gpu.py" \
 "step rn50 300 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step rn50_nd0 300 env FLAGS_native_dispatch=0 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step overhead 120 python -u benchmarks/dispatch_overhead.py" \
 "step snprobe 240 python -u benchmarks/conv_sn_probe.py" \
 "step rn50_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn7 -o run -- python3 benchmarks/resnet50.py --batch 256 --steps 5 --warmup 2"
