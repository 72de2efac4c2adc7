set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step probe 300 python -u tools/r5/moe_leak_probe.py" \
 "step probe_nonative 300 env FLAGS_native_dispatch=0 python -u tools/r5/moe_leak_probe.py" \
 "step causal_nonative 300 env FLAGS_native_dispatch=0 python -u -m pytest tests/test_causality_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k ernie"
