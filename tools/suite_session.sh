set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step suite 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider"
