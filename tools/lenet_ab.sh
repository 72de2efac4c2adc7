cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
set -o pipefail
for b in 128 512; do
  timeout -k 10 150 python -u benchmarks/mnist_lenet.py --batch $b --steps 200 >> gpurun_out/lenet_ab.jsonl 2>>gpurun_out/lenet_err.log || exit $?
  PADDLE_AMD_CONVND=0 timeout -k 10 150 python -u benchmarks/mnist_lenet.py --batch $b --steps 200 | sed 's/}$/, "path": "miopen"}/' >> gpurun_out/lenet_ab.jsonl 2>>gpurun_out/lenet_err.log || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/lenet_prof -o lenet -- python3 benchmarks/mnist_lenet.py --batch 128 --steps 50 > gpurun_out/lenet_prof.log 2>&1
