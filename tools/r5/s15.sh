set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
S=tools/gpu_session.sh
bash $S "step prof15 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_moe15 -o run -- python3 benchmarks/train_lm.py --model ernie-moe-a3b-8l --grouped-experts --fp8-experts --micro-batch 8 --accum 4 --steps 2 --warmup 1 --pool 8"
