"""cos_sim, bilinear / nearest interpolation, conv_shift and lstm_unit kernels
(csrc/kernels/nnmisc.hip) against fp64 PyTorch expressions of the same ops,
forward and backward, fp32 and bf16."""
import pytest
import torch
import torch.nn.functional as F

from paddle_amd.ops import nnmisc

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("yrows", [1, 7])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_cos_sim(yrows, dtype):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(7, 3, 50, generator=g).to(dtype).double()
    y = torch.randn(yrows, 3, 50, generator=g).to(dtype).double()
    xr, yr = x.clone().requires_grad_(), y.clone().requires_grad_()
    x2, y2 = xr.reshape(7, -1), yr.reshape(yrows, -1)
    ref = (x2 * y2).sum(1, keepdim=True) / (x2.norm(dim=1, keepdim=True) * y2.norm(dim=1, keepdim=True))
    xd, yd = x.to(dtype).to(DEV).requires_grad_(), y.to(dtype).to(DEV).requires_grad_()
    out, xn, yn = nnmisc.cos_sim(xd, yd)
    tol = 1e-6 if dtype == torch.float32 else 2e-2
    assert _rel(out, ref) < tol
    assert _rel(xn, x2.norm(dim=1, keepdim=True)) < tol
    gy = torch.randn(7, 1, generator=g, dtype=torch.float64)
    ref.backward(gy)
    out.backward(gy.to(dtype).to(DEV))
    assert _rel(xd.grad, xr.grad) < (1e-5 if dtype == torch.float32 else 3e-2)
    assert _rel(yd.grad, yr.grad) < (1e-5 if dtype == torch.float32 else 3e-2)


@pytest.mark.parametrize("mode,align", [("bilinear", True), ("bilinear", False), ("nearest", False)])
@pytest.mark.parametrize("size", [(13, 9), (4, 3)])
def test_interpolate(mode, align, size):
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, 3, 7, 5, generator=g, dtype=torch.float64)
    xr = x.clone().requires_grad_()
    kw = {"align_corners": align} if mode == "bilinear" else {}
    ref = F.interpolate(xr, size, mode=mode, **kw)
    xd = x.float().to(DEV).requires_grad_()
    y = nnmisc.interpolate(xd, size[0], size[1], mode, align)
    assert _rel(y, ref) < 1e-6
    gy = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    ref.backward(gy)
    y.backward(gy.float().to(DEV))
    assert _rel(xd.grad, xr.grad) < 1e-6


def test_conv_shift():
    g = torch.Generator().manual_seed(2)
    x = torch.randn(4, 11, generator=g, dtype=torch.float64)
    y = torch.randn(4, 5, generator=g, dtype=torch.float64)
    xr, yr = x.clone().requires_grad_(), y.clone().requires_grad_()
    M, Nn = 11, 5
    idx = (torch.arange(M)[:, None] + torch.arange(Nn)[None, :] - (Nn - 1) // 2) % M
    ref = (xr[:, idx] * yr[:, None, :]).sum(-1)
    xd, yd = x.float().to(DEV).requires_grad_(), y.float().to(DEV).requires_grad_()
    out = nnmisc.conv_shift(xd, yd)
    assert _rel(out, ref) < 1e-6
    gy = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    ref.backward(gy)
    out.backward(gy.float().to(DEV))
    assert _rel(xd.grad, xr.grad) < 1e-6
    assert _rel(yd.grad, yr.grad) < 1e-6


@pytest.mark.parametrize("fb", [0.0, 1.0])
def test_lstm_unit(fb):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(5, 4 * 24, generator=g, dtype=torch.float64)
    cp = torch.randn(5, 24, generator=g, dtype=torch.float64)
    xr, cr = x.clone().requires_grad_(), cp.clone().requires_grad_()
    i, f, o, gg = xr.split(24, 1)
    c = torch.sigmoid(f + fb) * cr + torch.sigmoid(i) * torch.tanh(gg)
    h = torch.sigmoid(o) * torch.tanh(c)
    xd, cd = x.float().to(DEV).requires_grad_(), cp.float().to(DEV).requires_grad_()
    c2, h2 = nnmisc.lstm_unit(xd, cd, fb)
    assert _rel(c2, c) < 1e-6 and _rel(h2, h) < 1e-6
    gc = torch.randn(5, 24, generator=g, dtype=torch.float64)
    gh = torch.randn(5, 24, generator=g, dtype=torch.float64)
    (c * gc + h * gh).sum().backward()
    (c2 * gc.float().to(DEV) + h2 * gh.float().to(DEV)).sum().backward()
    assert _rel(xd.grad, xr.grad) < 1e-5
    assert _rel(cd.grad, cr.grad) < 1e-5


@pytest.mark.parametrize("soft", [False, True])
def test_cross_entropy_on_probabilities(soft):
    g = torch.Generator().manual_seed(4)
    p = torch.softmax(torch.randn(9, 7, generator=g, dtype=torch.float64), -1)
    if soft:
        lab = torch.softmax(torch.randn(9, 7, generator=g, dtype=torch.float64), -1)
        pr = p.clone().requires_grad_()
        ref = -(lab * torch.log(pr)).sum(-1, keepdim=True)
        labd = lab.float().to(DEV)
    else:
        lab = torch.randint(0, 7, (9, 1), generator=g)
        lab[3, 0] = -100  # ignored row
        pr = p.clone().requires_grad_()
        safe = lab.clamp_min(0)
        ref = torch.where(lab == -100, torch.zeros(9, 1, dtype=torch.float64), -torch.log(pr.gather(1, safe)))
        labd = lab.to(DEV)
    pd = p.float().to(DEV).requires_grad_()
    y = nnmisc.cross_entropy(pd, labd, soft, -100)
    assert _rel(y, ref) < 1e-6
    gy = torch.randn(9, 1, generator=g, dtype=torch.float64)
    ref.backward(gy)
    y.backward(gy.float().to(DEV))
    assert _rel(pd.grad, pr.grad) < 1e-6
