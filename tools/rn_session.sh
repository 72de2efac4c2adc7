set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step aten 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_aten_native_gpu.py tests/test_eager_engine_gpu.py tests/test_conv_gpu.py" \
 "step rn50 400 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step rn50_nd0 400 env FLAGS_native_dispatch=0 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step rn50_graph 400 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5 --graph" \
 "step eager_probe 300 env FLAGS_count_aten=1 python -u tools/eager_trace_probe.py" \
 "step rn50_prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn5 -o run -- python3 benchmarks/resnet50.py --batch 256 --steps 5 --warmup 2"
