cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u benchmarks/fluid_resnet50.py --batch 32 >> gpurun_out/fluid_resnet_ab.jsonl 2>gpurun_out/fr_err.log || exit $?
PADDLE_AMD_CONVND=0 timeout -k 10 300 python -u benchmarks/fluid_resnet50.py --batch 32 >> gpurun_out/fluid_resnet_ab.jsonl 2>>gpurun_out/fr_err.log || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/fr_prof -o fr -- python3 benchmarks/fluid_resnet50.py --batch 32 --steps 3 --warmup 1 > gpurun_out/fr_prof.log 2>&1
