set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step eager17 300 env FLAGS_strict_trace=1 python -u tools/eager_trace_probe.py" "step disp17 200 python -u benchmarks/dispatch_overhead.py"
