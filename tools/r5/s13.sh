set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
S=tools/gpu_session.sh
bash $S "step t13 400 python -u -m pytest tests/test_kernels_gpu.py -k rope_attention_packed tests/test_strict_native_models_gpu.py -v --timeout 200 --timeout-method thread -p no:cacheprovider" \
 "step prof13 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_moe13 -o run -- python3 benchmarks/train_lm.py --model ernie-moe-a3b-8l --grouped-experts --fp8-experts --micro-batch 8 --accum 4 --steps 2 --warmup 1 --pool 8"
