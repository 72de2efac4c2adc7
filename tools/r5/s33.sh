set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step suite33 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "step smoke33 300 python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "step bench33 400 python -u bench.py --gpus 1 --steps 20 --warmup 5" \
 "step strict33 300 python -u tools/r5/strict_models.py"
