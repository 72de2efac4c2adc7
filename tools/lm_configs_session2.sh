set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step gpt13b 600 python -u benchmarks/train_lm.py --model gpt3-13b --micro-batch 2 --accum 4 --steps 10 --warmup 2" \
 "step moe_bf16 500 python -u benchmarks/train_lm.py --model ernie-moe-a3b-8l --grouped-experts --micro-batch 8 --accum 4 --steps 10 --warmup 2" \
 "step moe_fp8 500 python -u benchmarks/train_lm.py --model ernie-moe-a3b-8l --grouped-experts --fp8-experts --micro-batch 8 --accum 4 --steps 10 --warmup 2" \
 "step moe_fp8_prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_moe8 -o run -- python3 benchmarks/train_lm.py --model ernie-moe-a3b-8l --grouped-experts --fp8-experts --micro-batch 8 --accum 4 --steps 2 --warmup 1" \
 "step gpt13b_prof 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpt13 -o run -- python3 benchmarks/train_lm.py --model gpt3-13b --micro-batch 2 --accum 4 --steps 2 --warmup 1"
