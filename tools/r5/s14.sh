set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
S=tools/gpu_session.sh
bash $S "step t14 500 python -u -m pytest tests/test_grouped_gpu.py tests/test_moe_route_native_gpu.py tests/test_strict_native_models_gpu.py -v --timeout 200 --timeout-method thread -p no:cacheprovider" \
 "step moe_bf16_14 400 python -u benchmarks/train_lm.py --model ernie-moe-a3b-8l --grouped-experts --micro-batch 8 --accum 4 --steps 8 --warmup 2 --pool 64" \
 "step moe_fp8_14 400 python -u benchmarks/train_lm.py --model ernie-moe-a3b-8l --grouped-experts --fp8-experts --micro-batch 8 --accum 4 --steps 8 --warmup 2 --pool 64" \
 "step moe_fp8w_14 400 env FLAGS_fp8_wgrad=1 python -u benchmarks/train_lm.py --model ernie-moe-a3b-8l --grouped-experts --fp8-experts --micro-batch 8 --accum 4 --steps 8 --warmup 2 --pool 64"
