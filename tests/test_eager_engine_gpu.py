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


def _traj(make, place, dtype, batches, opt_make, sd=None):
    paddle.set_device(place)
    try:
        model = make()
        if sd is not None:
            model.set_state_dict(sd)
        if place == "gpu":
            model.to(device="cuda", dtype=dtype)
        opt = opt_make(model.parameters())
        losses = []
        with no_torch_autograd():
            for x, y in batches:
                xx = paddle.to_tensor(x).astype(str(dtype).split(".")[-1])
                out = model(xx).astype("float32")
                loss = F.cross_entropy(out, paddle.to_tensor(y))
                loss.backward()
                opt.step()
                opt.clear_grad()
                losses.append(float(loss))
        return losses
    finally:
        paddle.set_device("cpu")


def _oracle(make, dtype, shape, opt_make, steps=3, rtol=1e-3, seed=3):
    """The same model, init and batches on the GPU (``dtype``) and in fp32 on the CPU:
    the per-step losses must agree to ``rtol`` (a trajectory, not "loss went down")."""
    _native.lib()
    paddle.seed(seed)
    ref_model = make()
    sd = {k: v.detach().clone() for k, v in ref_model.state_dict().items()}
    rs = np.random.RandomState(seed)
    batches = [(rs.randn(*shape).astype("float32"), (np.arange(shape[0]) % 10).astype("int64"))
               for _ in range(steps)]
    cpu = _traj(make, "cpu", torch.float32, batches, opt_make, sd)
    gpu = _traj(make, "gpu", dtype, batches, opt_make, sd)
    for a, b in zip(cpu, gpu):
        assert abs(a - b) <= rtol * abs(a), (cpu, gpu)
    return cpu, gpu


def test_lenet_fp32_gpu_trajectory_matches_cpu_fp32():
    _oracle(paddle.vision.models.LeNet, torch.float32, (16, 1, 28, 28),
            lambda ps: paddle.optimizer.Adam(learning_rate=2e-3, parameters=ps), rtol=1e-3)


def test_resnet18_fp32_nhwc_gpu_trajectory_matches_cpu_fp32():
    """fp32 on both sides: isolates kernel/engine errors from bf16 rounding."""
    import os

    if os.environ.get("FLAGS_strict_native") == "1":
        pytest.skip("fp32 NHWC conv / BN / pool run the vendor path (native kernels: bf16 NHWC, fp32 NCHW)")
    _oracle(lambda: paddle.vision.models.resnet18(num_classes=10, data_format="NHWC"), torch.float32,
            (16, 64, 64, 3), lambda ps: paddle.optimizer.Momentum(learning_rate=0.01, momentum=0.9, parameters=ps),
            rtol=5e-3)


def test_resnet18_bf16_nhwc_gpu_trajectory_matches_cpu_fp32():
    """AMP-O2 style: bf16 parameters/activations with fp32 master weights.  BN over
    16x2x2 values per channel in layer4 and bf16 rounding bound the agreement, so two
    steps at 3e-2 (the first step is a pure forward check)."""
    _oracle(lambda: paddle.vision.models.resnet18(num_classes=10, data_format="NHWC"), torch.bfloat16,
            (16, 64, 64, 3),
            lambda ps: paddle.optimizer.Momentum(learning_rate=0.01, momentum=0.9, parameters=ps,
                                                 multi_precision=True),
            steps=2, rtol=3e-2)
