set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step moe_native 400 python -u -m pytest tests/test_moe_route_native_gpu.py tests/test_grouped_gpu.py tests/test_strict_native_models_gpu.py -v --timeout 200 --timeout-method thread -p no:cacheprovider" \
 "step strict_ernie 200 python -u tools/r5/strict_models.py ernie" \
 "step moe_bf16 400 python -u benchmarks/train_lm.py --model ernie-moe-a3b-8l --grouped-experts --micro-batch 8 --accum 4 --steps 8 --warmup 2 --pool 64" \
 "step moe_fp8 400 python -u benchmarks/train_lm.py --model ernie-moe-a3b-8l --grouped-experts --fp8-experts --micro-batch 8 --accum 4 --steps 8 --warmup 2 --pool 64" \
 "step gpt13b 500 python -u benchmarks/train_lm.py --model gpt3-13b --micro-batch 2 --accum 4 --steps 8 --warmup 2 --fixed-batch"
