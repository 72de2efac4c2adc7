set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step aten 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_aten_native_gpu.py" \
 "step native_book 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_native_engine_book_gpu.py tests/test_native_engine_gpu.py" \
 "step census_ops 600 env FLAGS_count_aten=1 PA_ATEN_REPORT=gpurun_out/census_ops.json python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_fluidk_gpu.py tests/test_eager_engine_gpu.py" \
 "step eager_probe 300 env FLAGS_count_aten=1 python -u tools/eager_trace_probe.py"
