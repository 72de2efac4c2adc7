set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step t20 600 python -u -m pytest tests/test_fastops_gpu.py tests/test_aten_native_gpu.py tests/test_eager_engine_gpu.py tests/test_ops_gpu.py tests/test_fluidk_gpu.py -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "step disp20 200 python -u benchmarks/dispatch_overhead.py"
