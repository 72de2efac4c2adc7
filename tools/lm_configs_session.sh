set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step overhead 120 python -u benchmarks/dispatch_overhead.py" \
 "step rn50_graph 400 env FLAGS_allocator_strategy=torch_caching python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5 --graph" \
 "step newtests 900 python -u -m pytest -q --timeout 600 --timeout-method thread tests/test_strict_native_gpu.py tests/test_runtime_trace_gpu.py tests/test_native_engine_book_gpu.py tests/test_aten_native_gpu.py tests/test_eager_engine_gpu.py" \
 "step gpt13b 600 python -u benchmarks/train_lm.py --model gpt3-13b --micro-batch 2 --accum 4 --steps 10 --warmup 2" \
 "step moe_bf16 500 python -u benchmarks/train_lm.py --model ernie-moe-a3b-8l --grouped-experts --micro-batch 8 --accum 4 --steps 10 --warmup 2" \
 "step moe_fp8 500 python -u benchmarks/train_lm.py --model ernie-moe-a3b-8l --grouped-experts --fp8-experts --micro-batch 8 --accum 4 --steps 10 --warmup 2"
