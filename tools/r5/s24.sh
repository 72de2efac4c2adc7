set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step suite24 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "step smoke24 300 python -u -c 'import __graft_entry__ as g; g.smoke()'" \
 "step bench24 400 python -u bench.py --gpus 1 --steps 20 --warmup 5" \
 "step gpt24 400 python -u benchmarks/train_lm.py --model gpt3-13b --micro-batch 2 --accum 4 --steps 8 --warmup 2 --fixed-batch" \
 "step moe24 400 python -u benchmarks/train_lm.py --model ernie-moe-a3b-8l --grouped-experts --micro-batch 8 --accum 4 --steps 8 --warmup 2 --pool 64" \
 "step moe8_24 400 python -u benchmarks/train_lm.py --model ernie-moe-a3b-8l --grouped-experts --fp8-experts --micro-batch 8 --accum 4 --steps 8 --warmup 2 --pool 64"
