"""paddle.* DyGraph API on the HIP device: fused optimizer kernels vs CPU math,
bf16 multi-precision training, flash-attention MHA path, LeNet/ResNet steps."""
import pytest
import torch

import paddle
import paddle.nn as nn
import paddle.nn.functional as F

pytestmark = pytest.mark.gpu


def test_adam_fused_kernel_matches_cpu():
    torch.manual_seed(0)
    w = torch.randn(1000)
    gs = [torch.randn(1000) for _ in range(3)]
    res = []
    for dev in ("cpu", "cuda"):
        p = nn.Linear(2, 2).weight
        p.data = w.clone().to(dev)
        opt = paddle.optimizer.AdamW(learning_rate=0.05, parameters=[p], weight_decay=0.1)
        for g in gs:
            p.grad = g.to(dev)
            opt.step()
        res.append(p.detach().cpu())
    assert torch.allclose(res[0], res[1], atol=1e-5)


def test_momentum_bf16_multi_precision():
    p = nn.Linear(2, 2).weight
    p.data = torch.ones(4096, device="cuda", dtype=torch.bfloat16)
    opt = paddle.optimizer.Momentum(learning_rate=1e-3, momentum=0.9, parameters=[p], multi_precision=True)
    for _ in range(10):
        p.grad = torch.full_like(p, 0.01)
        opt.step()
    master = opt._master[id(p)]
    assert master.dtype == torch.float32
    # 10 tiny steps accumulate in fp32 (a bf16-only update would stall at 1.0)
    assert float(master[0]) < 1.0 - 4e-4


def test_lenet_trains_on_gpu():
    paddle.seed(0)
    model = paddle.vision.models.LeNet().cuda()
    opt = paddle.optimizer.Adam(learning_rate=2e-3, parameters=model.parameters())
    ds = paddle.vision.datasets.MNIST(mode="train", num_samples=512)
    first = last = None
    for _ in range(3):
        for x, y in paddle.io.DataLoader(ds, batch_size=64, shuffle=True, device="cuda"):
            loss = F.cross_entropy(model(x), y)
            loss.backward()
            opt.step()
            opt.clear_grad()
            first = float(loss) if first is None else first
            last = float(loss)
    assert last < 0.5 * first


def test_mha_flash_path_bf16():
    paddle.seed(0)
    mha = nn.MultiHeadAttention(256, 4).cuda().to(torch.bfloat16)
    x = torch.randn(2, 64, 256, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    a = mha(x, is_causal=True)
    b = mha(x, attn_mask=torch.ones(64, 64, dtype=torch.bool, device="cuda").tril())
    assert (a.float() - b.float()).abs().max() < 3e-2
    a.float().sum().backward()
    assert x.grad is not None


def test_resnet50_nhwc_bf16_step():
    paddle.seed(0)
    m = paddle.vision.models.resnet50(num_classes=102, data_format="NHWC").cuda()
    opt = paddle.optimizer.Momentum(0.1, 0.9, parameters=m.parameters())
    m, opt = paddle.amp.decorate(m, opt, level="O2")
    x = torch.randn(8, 224, 224, 3, device="cuda", dtype=torch.bfloat16)
    y = torch.randint(0, 102, (8, 1), device="cuda")
    loss = F.cross_entropy(m(x).float(), y)
    loss.backward()
    opt.step()
    assert torch.isfinite(loss)
