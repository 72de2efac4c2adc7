#!/usr/bin/env python3
"""ResNet-50 training throughput (images/s), DyGraph, one MI355X.

Reference number: 105.84 images/s, Fluid ResNet-50 on Flowers102 (224x224, 102
classes), 1x TITAN X Pascal (doc/fluid/new_docs/advanced_usage/benchmark.rst:117;
model benchmark/fluid/models/resnet.py).  Same model/shape here with synthetic
data and random init; Momentum(0.9) + L2 1e-4 like the reference benchmark.

MI355X configuration: NHWC activations (MIOpen NHWC MFMA convolutions, no
layout transposes), ``--amp O2`` = bf16 parameters/activations with fp32 master
weights in the fused Momentum kernel and fp32 BatchNorm statistics.
"""
import argparse
import json
import sys
import os
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--amp", default="O2", choices=["O0", "O1", "O2"])
    ap.add_argument("--data-format", default="NHWC")
    ap.add_argument("--classes", type=int, default=102)
    ap.add_argument("--graph", action="store_true",
                    help="capture one whole training step (forward, backward, Momentum) into a HIP graph "
                         "after warm-up and replay it: no host launch overhead per kernel")
    a = ap.parse_args()

    import paddle_amd as paddle
    from paddle_amd import nn

    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    if dev.type == "cuda" and os.environ.get("PA_SET_DEVICE", "0") == "1":
        paddle.set_device("gpu")
    paddle.seed(0)
    model = paddle.vision.models.resnet50(num_classes=a.classes, data_format=a.data_format).to(dev)
    opt = paddle.optimizer.Momentum(learning_rate=0.1, momentum=0.9, parameters=model.parameters(),
                                    weight_decay=paddle.optimizer.L2Decay(1e-4))
    if a.amp == "O2":
        model, opt = paddle.amp.decorate(model, opt, level="O2", dtype="bfloat16")
    loss_fn = nn.CrossEntropyLoss()
    B = a.batch
    shape = (B, 224, 224, 3) if a.data_format == "NHWC" else (B, 3, 224, 224)
    dt = torch.bfloat16 if a.amp == "O2" else torch.float32
    x = torch.randn(shape, device=dev, dtype=dt)
    y = torch.randint(0, a.classes, (B, 1), device=dev)

    def step():
        if a.amp == "O1":
            with paddle.amp.auto_cast(dtype="bfloat16"):
                out = model(x)
        else:
            out = model(x)
        loss = loss_fn(out.float() if out.dtype != torch.float32 else out, y)
        loss.backward()
        opt.step()
        opt.clear_grad(set_to_zero=False)
        return loss

    run = step
    if a.graph and dev.type == "cuda":
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(max(a.warmup, 2)):
                step()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        import gc

        gc.collect()
        gc.disable()  # no pinned-buffer frees (hipHostFree) from the collector mid-capture
        # relaxed: HIP refuses hipMalloc while a stream captures in global / thread_local
        # mode (hipErrorStreamCaptureUnsupported), and the graph pool must grow on the
        # first capture of a step this size (profiles/r4_rn50_graph_capture.md)
        try:
            with torch.cuda.graph(g, capture_error_mode=os.environ.get("PA_CAPTURE_MODE", "relaxed")):
                static_loss = step()
        finally:
            gc.enable()

        def run():
            g.replay()
            return static_loss
    for _ in range(a.warmup):
        run()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = run()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt_s = time.perf_counter() - t0
    ips = a.steps * B / dt_s
    print(json.dumps({"metric": "ResNet-50 train images/s (Flowers102 shape, synthetic)", "value": round(ips, 1),
                      "unit": "images/s", "batch": B, "steps": a.steps, "amp": a.amp, "data_format": a.data_format,
                      "ms_per_step": round(1000 * dt_s / a.steps, 2), "baseline": 105.84, "hip_graph": a.graph,
                      "vs_baseline": round(ips / 105.84, 2), "loss": float(loss)}))


if __name__ == "__main__":
    main()
