#!/bin/bash
# ResNet-50 --graph with relaxed capture vs eager; native-engine GPU tests
mkdir -p gpurun_out
run() { local name=$1; shift; echo "=== $name: $*"; timeout -k 10 300 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -3 gpurun_out/$name.log; return $rc; }
run native_gpu python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_native_engine_gpu.py tests/test_hip_graph_gpu.py &&
run rn50_graph python -u benchmarks/resnet50.py --batch 256 --steps 30 --warmup 5 --graph &&
run rn50 python -u benchmarks/resnet50.py --batch 256 --steps 30 --warmup 5 &&
run rn50_graph2 python -u benchmarks/resnet50.py --batch 256 --steps 30 --warmup 5 --graph
