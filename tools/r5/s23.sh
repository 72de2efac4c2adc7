set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step norm23 300 python -u benchmarks/norm_bwd_ab.py" \
 "step t23 300 python -u -m pytest tests/test_kernels_gpu.py -k norm -q --timeout 200 --timeout-method thread -p no:cacheprovider"
