set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
S=tools/gpu_session.sh
bash $S "step abA1 300 python -u bench.py --steps 10 --warmup 3" \
 "step abB1 300 env FLAGS_fastops=0 PA_NORM_BWD_RPB=4 FLAGS_gemm_splitk=0 python -u bench.py --steps 10 --warmup 3" \
 "step abA2 300 python -u bench.py --steps 10 --warmup 3" \
 "step abB2 300 env FLAGS_fastops=0 PA_NORM_BWD_RPB=4 FLAGS_gemm_splitk=0 python -u bench.py --steps 10 --warmup 3"
