set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
S=tools/gpu_session.sh
bash $S "step suite16 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "step smoke16 300 python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "step eager16 300 python -u tools/eager_trace_probe.py"
