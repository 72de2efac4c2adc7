set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step rnA1 300 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step rnB1 300 env PA_BN_APPLY=0 PA_BN_DX=0 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step rnC1 300 env PA_BN_DX=0 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step rnA2 300 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step rnB2 300 env PA_BN_APPLY=0 PA_BN_DX=0 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5" \
 "step rnC2 300 env PA_BN_DX=0 python -u benchmarks/resnet50.py --batch 256 --steps 20 --warmup 5"
