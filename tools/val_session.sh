set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step newtests 900 python -u -m pytest -q --timeout 600 --timeout-method thread tests/test_strict_native_gpu.py tests/test_runtime_trace_gpu.py tests/test_native_engine_book_gpu.py tests/test_aten_native_gpu.py"
