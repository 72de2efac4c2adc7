"""Remaining op-library kernels (csrc/kernels/misc.hip) against fp32 / exact
references: one_hot, pad2d (constant / reflect / edge, NCHW / NHWC, backward),
cross-channel LRN (fwd + bwd vs autograd of the reference formula), LoD row_conv
(fwd + dx + dW), argsort, accuracy, concat / split (with backward)."""
import pytest
import torch
import torch.nn.functional as F

from paddle_amd.ops import oplib

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_one_hot():
    x = torch.tensor([0, 3, 2, 3, 1], device=DEV)
    out = oplib.one_hot(x, 4)
    assert torch.equal(out.cpu(), F.one_hot(x.cpu(), 4).float())
    with pytest.raises(ValueError):
        oplib.one_hot(torch.tensor([5], device=DEV), 4)


@pytest.mark.parametrize("mode", ["constant", "reflect", "edge"])
@pytest.mark.parametrize("nhwc", [False, True])
def test_pad2d_fwd_bwd(mode, nhwc):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 3, 5, 6, generator=g)
    pads = (1, 2, 3, 1)  # top, bottom, left, right
    xd = (x.permute(0, 2, 3, 1).contiguous() if nhwc else x).to(DEV).requires_grad_(True)
    y = oplib.pad2d_op(xd, pads, mode, 0.5, nhwc)
    tmode = {"constant": "constant", "reflect": "reflect", "edge": "replicate"}[mode]
    xr = x.clone().requires_grad_(True)
    kw = {"value": 0.5} if mode == "constant" else {}
    ref = F.pad(xr, (pads[2], pads[3], pads[0], pads[1]), mode=tmode, **kw)
    got = y.permute(0, 3, 1, 2) if nhwc else y
    torch.testing.assert_close(got.cpu(), ref.detach(), rtol=0, atol=0)
    gy = torch.randn(ref.shape, generator=g)
    ref.backward(gy)
    (got * (gy.to(DEV))).sum().backward()
    gx = xd.grad.permute(0, 3, 1, 2) if nhwc else xd.grad
    torch.testing.assert_close(gx.cpu(), xr.grad, rtol=1e-5, atol=1e-5)


def _lrn_ref(x, n, k, a, b):
    C = x.shape[1]
    pre = (n - 1) // 2
    sq = x * x
    mids = []
    for c in range(C):
        lo, hi = max(0, c - pre), min(C, c - pre + n)
        mids.append(k + a * sq[:, lo:hi].sum(1))
    mid = torch.stack(mids, 1)
    return x * mid.pow(-b), mid


@pytest.mark.parametrize("n", [5, 4])
def test_lrn_fwd_bwd(n):
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, 7, 4, 5, generator=g, dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    ref, mid_ref = _lrn_ref(xr, n, 2.0, 1e-2, 0.75)
    xd = x.float().to(DEV).requires_grad_(True)
    out, mid = oplib.lrn_op(xd, n, 2.0, 1e-2, 0.75)
    torch.testing.assert_close(out.double().cpu(), ref.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(mid.double().cpu(), mid_ref.detach(), rtol=1e-5, atol=1e-6)
    gy = torch.randn(x.shape, generator=g, dtype=torch.float64)
    ref.backward(gy)
    (out * gy.float().to(DEV)).sum().backward()
    torch.testing.assert_close(xd.grad.double().cpu(), xr.grad, rtol=1e-4, atol=1e-5)


def test_row_conv_fwd_bwd():
    g = torch.Generator().manual_seed(2)
    off = [0, 3, 8, 9, 15]
    x = torch.randn(15, 6, generator=g, dtype=torch.float64)
    w = torch.randn(3, 6, generator=g, dtype=torch.float64)
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    outs = []
    for s, e in zip(off[:-1], off[1:]):
        seq = xr[s:e]
        o = torch.zeros_like(seq)
        for k in range(w.shape[0]):
            if k < e - s:
                o = o + F.pad(seq[k:] * wr[k], (0, 0, 0, k))
        outs.append(o)
    ref = torch.cat(outs)
    xd = x.float().to(DEV).requires_grad_(True)
    wd = w.float().to(DEV).requires_grad_(True)
    out = oplib.row_conv_op(xd, wd, off)
    torch.testing.assert_close(out.double().cpu(), ref.detach(), rtol=1e-5, atol=1e-5)
    gy = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    ref.backward(gy)
    (out * gy.float().to(DEV)).sum().backward()
    torch.testing.assert_close(xd.grad.double().cpu(), xr.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(wd.grad.double().cpu(), wr.grad, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("n", [1, 7, 64, 1000, 2048])
def test_argsort_rows(n):
    g = torch.Generator().manual_seed(n)
    x = torch.randint(-50, 50, (5, n), generator=g).float()  # ties: indices must be ascending within ties
    v, i = oplib.argsort_op(x.to(DEV))
    rv, ri = torch.sort(x, dim=-1, stable=True)
    assert torch.equal(v.cpu(), rv) and torch.equal(i.cpu(), ri)


def test_accuracy():
    ind = torch.tensor([[1, 2], [0, 3], [4, 4], [2, 0]], device=DEV)
    lab = torch.tensor([[2], [1], [4], [0]], device=DEV)
    acc, correct, total = oplib.accuracy_op(ind, lab)
    assert abs(acc.item() - 0.75) < 1e-7 and correct.item() == 3 and total.item() == 4


@pytest.mark.parametrize("axis", [0, 1, 2])
def test_concat_split_with_grad(axis):
    g = torch.Generator().manual_seed(3)
    xs = [torch.randn(*(s if d == axis else base for d, base in enumerate((4, 5, 6))), generator=g)
          for s in (2, 3, 1)]
    xd = [x.to(DEV).requires_grad_(True) for x in xs]
    out = oplib.concat_op(xd, axis)
    ref = torch.cat(xs, axis)
    assert torch.equal(out.cpu(), ref)
    parts = oplib.split_op(out, [x.shape[axis] for x in xs], axis)
    for p, x in zip(parts, xs):
        assert torch.equal(p.cpu(), x)
    gy = torch.randn(ref.shape, generator=g)
    (out * gy.to(DEV)).sum().backward()
    for x, xdd, gg in zip(xs, xd, torch.split(gy, [x.shape[axis] for x in xs], axis)):
        assert torch.equal(xdd.grad.cpu(), gg)
