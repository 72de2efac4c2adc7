#!/usr/bin/env python3
"""ResNet-50 / VGG-16 inference through the inference library (AnalysisPredictor):
a Fluid program saved with save_inference_model, IR passes (conv+BN folding, fc
fusion), optional bf16 weights and HIP-graph replay -- the reference's
paddle/contrib/float16/float16_benchmark.md rows (bs 64: ResNet-50 67.93 ms fp32 /
33.20 ms fp16; VGG-16 178.95 / 60.23 ms on V100) measured the way a deployment
calls it: ``predictor.run([PaddleTensor(numpy batch)])``, host input included.

Networks follow benchmark/fluid/models/resnet.py (conv_bn_layer / shortcut /
bottleneck, ImageNet depth 50) and the VGG-16 of paddle/contrib/float16 (conv
groups + 2 x fc 4096); random weights, synthetic images.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

BASE = {("resnet50", "fp32"): 67.93, ("resnet50", "bf16"): 33.20, ("vgg16", "fp32"): 178.95,
        ("vgg16", "bf16"): 60.23}


def resnet50(fluid, img, class_dim=1000):
    def conv_bn(x, ch, k, s, p, act="relu"):
        c = fluid.layers.conv2d(input=x, num_filters=ch, filter_size=k, stride=s, padding=p, bias_attr=False)
        return fluid.layers.batch_norm(input=c, act=act)

    def shortcut(x, ch_out, s):
        return conv_bn(x, ch_out, 1, s, 0, None) if x.shape[1] != ch_out else x

    def bottleneck(x, ch, s):
        short = shortcut(x, ch * 4, s)
        y = conv_bn(x, ch, 1, s, 0)
        y = conv_bn(y, ch, 3, 1, 1)
        y = conv_bn(y, ch * 4, 1, 1, 0, None)
        return fluid.layers.relu(fluid.layers.elementwise_add(short, y))

    x = conv_bn(img, 64, 7, 2, 3)
    x = fluid.layers.pool2d(x, pool_size=3, pool_stride=2, pool_padding=1, pool_type="max")
    for ch, n, s in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
        for i in range(n):
            x = bottleneck(x, ch, s if i == 0 else 1)
    x = fluid.layers.pool2d(x, pool_type="avg", global_pooling=True)
    return fluid.layers.fc(input=x, size=class_dim, act="softmax")


def vgg16(fluid, img, class_dim=1000):
    x = img
    for nf, n in ((64, 2), (128, 2), (256, 3), (512, 3), (512, 3)):
        for _ in range(n):
            x = fluid.layers.conv2d(input=x, num_filters=nf, filter_size=3, padding=1, act="relu")
        x = fluid.layers.pool2d(x, pool_size=2, pool_stride=2, pool_type="max")
    x = fluid.layers.fc(input=x, size=4096, act="relu")
    x = fluid.layers.fc(input=x, size=4096, act="relu")
    return fluid.layers.fc(input=x, size=class_dim, act="softmax")


def save_model(name, d):
    import paddle_amd.fluid as fluid
    from paddle_amd.framework import core

    main, startup = fluid.Program(), fluid.Program()
    main.random_seed = startup.random_seed = 7
    with fluid.program_guard(main, startup):
        img = fluid.layers.data(name="img", shape=[3, 224, 224], dtype="float32")
        out = (resnet50 if name == "resnet50" else vgg16)(fluid, img)
    exe = fluid.Executor(fluid.CPUPlace())
    with fluid.executor.scope_guard(core.Scope()):
        exe.run(startup)
        fluid.io.save_inference_model(d, ["img"], [out], exe, main_program=main)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="resnet50,vgg16")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    from paddle_amd import inference

    x = np.random.RandomState(0).rand(a.batch, 3, 224, 224).astype("float32")
    for name in a.models.split(","):
        with tempfile.TemporaryDirectory() as d:
            save_model(name, d)
            for prec, graph in (("fp32", False), ("bf16", False), ("bf16", True)):
                cfg = inference.AnalysisConfig(model_dir=d, use_gpu=torch.cuda.is_available())
                if prec == "bf16":
                    cfg.enable_bf16()
                if graph:
                    cfg.enable_hip_graph()
                pred = inference.create_paddle_predictor(cfg)
                inp = [inference.PaddleTensor(x, name="img")]
                for _ in range(a.warmup):
                    out = pred.run(inp)
                t0 = time.perf_counter()
                for _ in range(a.iters):
                    out = pred.run(inp)          # returns host arrays: includes the D2H sync
                dt = (time.perf_counter() - t0) / a.iters * 1e3
                base = BASE[(name, prec)]
                print(json.dumps({"bench": f"predictor_{name}", "precision": prec, "hip_graph": graph,
                                  "batch": a.batch, "ms_per_batch": round(dt, 2), "baseline_ms": base,
                                  "speedup_vs_baseline": round(base / dt, 2),
                                  "passes": pred.pass_stats if hasattr(pred, "pass_stats") else None,
                                  "out_sum": float(out[0].as_ndarray().sum())}), flush=True)


if __name__ == "__main__":
    main()
