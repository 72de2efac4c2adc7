set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
S=tools/gpu_session.sh
bash $S "step prof21 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpt21 -o run -- python3 benchmarks/train_lm.py --model gpt3-13b --micro-batch 2 --accum 4 --steps 2 --warmup 1 --fixed-batch"
