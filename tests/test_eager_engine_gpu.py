"""The eager engine on the GPU: DyGraph LeNet (BASELINE config 1 on CUDAPlace) and a
ResNet-tiny bf16 NHWC step train with torch.autograd patched to raise, through the
hand-written HIP conv / BN / pool / GEMM / softmax-CE kernels (each recorded as one
grad node with its own backward kernels), and no op taking the fallback."""
import numpy as np
import pytest
import torch

import paddle
import paddle.nn.functional as F
from paddle_amd.ops import _native

from test_eager_engine_cpu import no_torch_autograd

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")]


def test_lenet_dygraph_gpu_trains_without_torch_autograd():
    _native.lib()
    paddle.seed(3)
    paddle.set_device("gpu")
    try:
        model = paddle.vision.models.LeNet()
        model.to("cuda")
        opt = paddle.optimizer.Adam(learning_rate=2e-3, parameters=model.parameters())
        ds = paddle.vision.datasets.MNIST(mode="train", num_samples=384)
        first = last = None
        with no_torch_autograd():
            for _ in range(2):
                for img, label in paddle.io.DataLoader(ds, batch_size=64, shuffle=True):
                    img, label = img.cuda(), label.cuda()
                    loss = F.cross_entropy(model(img), label)
                    loss.backward()
                    opt.step()
                    opt.clear_grad()
                    first = float(loss) if first is None else first
                    last = float(loss)
        assert last < first * 0.6, (first, last)
    finally:
        paddle.set_device("cpu")


def test_resnet_tiny_bf16_nhwc_gpu_without_torch_autograd():
    _native.lib()
    paddle.seed(0)
    paddle.set_device("gpu")
    try:
        model = paddle.vision.models.resnet18(num_classes=10, data_format="NHWC")
        model.to(device="cuda", dtype=torch.bfloat16)
        opt = paddle.optimizer.Momentum(learning_rate=0.05, momentum=0.9, parameters=model.parameters())
        x = paddle.randn([8, 32, 32, 3]).astype("bfloat16")
        y = paddle.to_tensor(np.arange(8) % 10)
        losses = []
        with no_torch_autograd():
            for _ in range(5):
                loss = F.cross_entropy(model(x).astype("float32"), y)
                loss.backward()
                opt.step()
                opt.clear_grad()
                losses.append(float(loss))
        assert losses[-1] < losses[0], losses
    finally:
        paddle.set_device("cpu")
