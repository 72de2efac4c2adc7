set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
S=tools/gpu_session.sh
bash $S "step bnab 300 python -u benchmarks/bn_apply_ab.py" \
 "step t26 400 python -u -m pytest tests/test_grouped_gpu.py tests/test_eager_engine_gpu.py tests/test_aten_native_gpu.py tests/test_fastops_gpu.py -q --timeout 200 --timeout-method thread -p no:cacheprovider" \
 "step moe26 400 python -u benchmarks/train_lm.py --model ernie-moe-a3b-8l --grouped-experts --micro-batch 8 --accum 4 --steps 8 --warmup 2 --pool 64" \
 "step moe8_26 400 python -u benchmarks/train_lm.py --model ernie-moe-a3b-8l --grouped-experts --fp8-experts --micro-batch 8 --accum 4 --steps 8 --warmup 2 --pool 64" \
 "step rn26 300 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step rn26prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rn26 -o run -- python3 benchmarks/resnet50.py --batch 256 --steps 5 --warmup 2"
