#!/usr/bin/env python3
"""Fluid static-graph ResNet-50 training (NCHW fp32, the reference's
benchmark/fluid/models/resnet.py network: conv-bn stem, bottleneck stages
[3, 4, 6, 3], global avg pool, fc softmax), synthetic images / labels.  On the
GPU every conv / BN / pool / fc runs through the Fluid operators' native kernels
(convnd.hip + the fp32 MFMA GEMM); ``PADDLE_AMD_CONVND=0`` routes them to
MIOpen / hipBLASLt instead for an A/B.  Prints one JSON line."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import paddle_amd.fluid as fluid  # noqa: E402


def conv_bn(x, ch, k, stride=1, act="relu"):
    c = fluid.layers.conv2d(x, ch, k, stride=stride, padding=(k - 1) // 2, bias_attr=False)
    return fluid.layers.batch_norm(c, act=act)


def bottleneck(x, ch, stride):
    short = conv_bn(x, ch * 4, 1, stride, act=None) if stride != 1 or x.shape[1] != ch * 4 else x
    y = conv_bn(x, ch, 1)
    y = conv_bn(y, ch, 3, stride)
    y = conv_bn(y, ch * 4, 1, act=None)
    return fluid.layers.relu(fluid.layers.elementwise_add(short, y))


def resnet50(img, classes):
    x = conv_bn(img, 64, 7, 2)
    x = fluid.layers.pool2d(x, 3, "max", 2, pool_padding=1)
    for i, (n, ch) in enumerate(zip([3, 4, 6, 3], [64, 128, 256, 512])):
        for j in range(n):
            x = bottleneck(x, ch, 2 if j == 0 and i > 0 else 1)
    x = fluid.layers.pool2d(x, 7, "avg", global_pooling=True)
    return fluid.layers.fc(x, classes, act="softmax")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--size", type=int, default=224)
    a = ap.parse_args()
    main_p, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main_p, startup):
        img = fluid.layers.data("img", [3, a.size, a.size])
        lbl = fluid.layers.data("label", [1], dtype="int64")
        pred = resnet50(img, 1000)
        loss = fluid.layers.mean(fluid.layers.cross_entropy(pred, lbl))
        fluid.optimizer.Momentum(0.01, 0.9).minimize(loss)
    place = fluid.CUDAPlace(0)
    exe = fluid.Executor(place)
    exe.run(startup)
    rs = np.random.RandomState(0)
    x = rs.randn(a.batch, 3, a.size, a.size).astype("float32")
    y = rs.randint(0, 1000, (a.batch, 1)).astype("int64")
    import torch

    for _ in range(a.warmup):
        exe.run(main_p, feed={"img": x, "label": y}, fetch_list=[loss])
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(a.steps):
        out = exe.run(main_p, feed={"img": x, "label": y}, fetch_list=[loss])
    torch.cuda.synchronize()
    dt = (time.time() - t0) / a.steps
    print(json.dumps({"metric": "Fluid ResNet-50 train images/s (NCHW fp32)", "value": round(a.batch / dt, 1),
                      "batch": a.batch, "ms_per_step": round(dt * 1e3, 2), "loss": float(np.array(out[0]).ravel()[0]),
                      "path": "native" if os.environ.get("PADDLE_AMD_CONVND", "1") != "0" else "miopen+hipblaslt"}),
          flush=True)


if __name__ == "__main__":
    main()
