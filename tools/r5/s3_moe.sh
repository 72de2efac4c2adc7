set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step causal 300 python -u -m pytest tests/test_causality_gpu.py -v --timeout 200 --timeout-method thread -p no:cacheprovider" \
 "step fa_gqa 300 python -u -m pytest tests/test_kernels_gpu.py -v --timeout 200 --timeout-method thread -p no:cacheprovider -k 'flash_attention or rope_attention_packed'" \
 "step moe_pool64 400 python -u benchmarks/train_lm.py --model ernie-moe-a3b-8l --grouped-experts --micro-batch 8 --accum 4 --steps 8 --warmup 2 --pool 64" \
 "step moe_pool8 400 python -u benchmarks/train_lm.py --model ernie-moe-a3b-8l --grouped-experts --micro-batch 8 --accum 4 --steps 8 --warmup 2 --pool 8" \
 "step gpt_fixed 500 python -u benchmarks/train_lm.py --model gpt3-13b --micro-batch 2 --accum 4 --steps 8 --warmup 2 --fixed-batch"
