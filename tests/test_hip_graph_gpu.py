"""A whole DyGraph training step (NHWC bf16 ResNet-18 forward, eager-engine
backward, multi-tensor Momentum) captured into one HIP graph and replayed: the
parameters follow the eagerly-run copy of the same model and data (the capture
path of benchmarks/resnet50.py --graph; the Momentum descriptor table of the
graph's pool addresses is uploaded by a captured copy)."""
import copy

import numpy as np
import pytest
import torch

import paddle
import paddle.nn.functional as F
from paddle_amd.ops import _native

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")]


def test_resnet18_step_hip_graph_replay_matches_eager():
    _native.lib()
    paddle.seed(5)
    paddle.set_device("gpu")
    try:
        base = paddle.vision.models.resnet18(num_classes=10, data_format="NHWC")
        base.to(device="cuda", dtype=torch.bfloat16)
        models = [base, copy.deepcopy(base)]
        opts = [paddle.optimizer.Momentum(learning_rate=0.01, momentum=0.9, parameters=m.parameters())
                for m in models]
        x = paddle.to_tensor(np.random.RandomState(0).randn(8, 32, 32, 3).astype("float32")).astype("bfloat16")
        y = paddle.to_tensor(np.arange(8) % 10)

        def step(i):
            loss = F.cross_entropy(models[i](x).astype("float32"), y)
            loss.backward()
            opts[i].step()
            opts[i].clear_grad(set_to_zero=False)
            return loss

        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                step(0)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            static_loss = step(0)
        # capture records without executing: model 0 has taken the 2 warm-up steps;
        # 3 replays make 5, as 5 eager steps of model 1
        for _ in range(3):
            g.replay()
        for _ in range(5):
            step(1)
        torch.cuda.synchronize()
        worst = 0.0
        for p0, p1 in zip(models[0].parameters(), models[1].parameters()):
            a, b = p0.float(), p1.float()
            worst = max(worst, float((a - b).abs().max() / (b.abs().max() + 1e-6)))
        assert worst < 2e-2, worst
        assert torch.isfinite(static_loss).all()
    finally:
        paddle.set_device("cpu")
