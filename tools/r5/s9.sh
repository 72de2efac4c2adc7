set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step native_ctl 400 python -u -m pytest tests/test_native_engine_control_gpu.py tests/test_lm_head_padded_gpu.py -v --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "step zero3_trace 300 env PA_TRACE_OUT=gpurun_out/zero3_overlap_trace.json python -u -m pytest tests/test_zero3_overlap_trace_gpu.py -v --timeout 280 --timeout-method thread -p no:cacheprovider" \
 "step strict_models 400 python -u tools/r5/strict_models.py" \
 "step norm_ab 300 python -u benchmarks/norm_bwd_ab.py"
