#!/usr/bin/env python3
"""Fluid static-graph MNIST LeNet training throughput (BASELINE.md parity floor:
19710.90 samples/s, Fluid 0.12 on 1x TITAN X Pascal, benchmark.rst:115).

Synthetic 28x28 images / random labels (no dataset download here).  The timed
region is full training steps (forward, backward, Adam) through fluid.Executor.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import paddle_amd.fluid as fluid  # noqa: E402
from paddle_amd.framework import core  # noqa: E402


def lenet(img, label):
    c1 = fluid.nets.simple_img_conv_pool(input=img, filter_size=5, num_filters=20, pool_size=2, pool_stride=2,
                                         act="relu")
    c2 = fluid.nets.simple_img_conv_pool(input=c1, filter_size=5, num_filters=50, pool_size=2, pool_stride=2,
                                         act="relu")
    pred = fluid.layers.fc(input=c2, size=10, act="softmax")
    loss = fluid.layers.mean(fluid.layers.cross_entropy(input=pred, label=label))
    return loss, fluid.layers.accuracy(input=pred, label=label)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--cpu", action="store_true")
    a = ap.parse_args()
    main_p, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main_p, startup):
        img = fluid.layers.data(name="img", shape=[1, 28, 28], dtype="float32")
        label = fluid.layers.data(name="label", shape=[1], dtype="int64")
        loss, acc = lenet(img, label)
        fluid.optimizer.Adam(learning_rate=0.001).minimize(loss)
    place = fluid.CPUPlace() if a.cpu else fluid.CUDAPlace(0)
    exe = fluid.Executor(place)
    exe.run(startup)
    rng = np.random.RandomState(0)
    import torch
    dev = place.torch_device()
    X = [core.LoDTensor(torch.from_numpy(rng.rand(a.batch, 1, 28, 28).astype("float32")).to(dev)) for _ in range(8)]
    Y = [core.LoDTensor(torch.from_numpy(rng.randint(0, 10, (a.batch, 1)).astype("int64")).to(dev)) for _ in range(8)]
    for i in range(a.warmup):
        exe.run(main_p, feed={"img": X[i % 8], "label": Y[i % 8]}, fetch_list=[], return_numpy=False)
    if not a.cpu:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        exe.run(main_p, feed={"img": X[i % 8], "label": Y[i % 8]}, fetch_list=[], return_numpy=False)
    (l,) = exe.run(main_p, feed={"img": X[0], "label": Y[0]}, fetch_list=[loss])
    if not a.cpu:
        torch.cuda.synchronize()
    el = time.perf_counter() - t0
    sps = a.batch * (a.steps + 1) / el
    print(json.dumps({"metric": "MNIST LeNet fluid train samples/s", "value": round(sps, 1), "unit": "samples/s",
                      "batch": a.batch, "steps": a.steps, "baseline": 19710.90, "vs_baseline": round(sps / 19710.90, 3),
                      "loss": float(l[0]), "place": str(place)}))


if __name__ == "__main__":
    main()
