set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step t12 500 python -u -m pytest tests/test_grouped_gpu.py tests/test_moe_route_native_gpu.py tests/test_strict_native_models_gpu.py -v --timeout 200 --timeout-method thread -p no:cacheprovider" \
 "step t12norm 300 python -u -m pytest tests/test_kernels_gpu.py -k norm -q --timeout 200 --timeout-method thread -p no:cacheprovider" \
 "step census12 300 python -u tools/r5/strict_models.py" \
 "step moe_fp8_12 400 python -u benchmarks/train_lm.py --model ernie-moe-a3b-8l --grouped-experts --fp8-experts --micro-batch 8 --accum 4 --steps 8 --warmup 2 --pool 64" \
 "step moe_bf16_12 400 python -u benchmarks/train_lm.py --model ernie-moe-a3b-8l --grouped-experts --micro-batch 8 --accum 4 --steps 8 --warmup 2 --pool 64" \
 "step bench12 400 python -u bench.py --steps 10 --warmup 3"
