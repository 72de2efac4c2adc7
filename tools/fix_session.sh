set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step fixtests 700 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_optimizer_ops_gpu.py tests/test_profiler_gpu.py tests/test_native_engine_book_gpu.py tests/test_eager_engine_gpu.py tests/test_strict_native_gpu.py" \
 "step profdbg_py 120 python -u tools/prof_auto_debug.py python" \
 "step profdbg_auto 120 python -u tools/prof_auto_debug.py auto"
