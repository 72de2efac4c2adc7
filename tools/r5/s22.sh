set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step t22 400 python -u -m pytest tests/test_gemm_splitk_gpu.py tests/test_gemm_gpu.py tests/test_models_gpu.py -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
 "step gpt22 500 python -u benchmarks/train_lm.py --model gpt3-13b --micro-batch 2 --accum 4 --steps 8 --warmup 2 --fixed-batch" \
 "step gpt22off 500 env FLAGS_gemm_splitk=0 python -u benchmarks/train_lm.py --model gpt3-13b --micro-batch 2 --accum 4 --steps 8 --warmup 2 --fixed-batch"
