set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step fixtests 300 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_native_engine_book_gpu.py tests/test_profiler_gpu.py" \
 "step profdbg_py 120 python -u tools/prof_auto_debug.py python" \
 "step profdbg_auto 120 python -u tools/prof_auto_debug.py auto" \
 "step dwprobe 240 python -u benchmarks/dw_vendor_probe.py" && \
bash tools/lm_configs_session2.sh
