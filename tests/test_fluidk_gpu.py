"""Fluid operator-library HIP kernels (csrc/kernels/fluid_ops.hip via
paddle_amd/ops/fluidk.py) against plain PyTorch fp32 references of the same op,
then the explicit grad ops through the Executor on CUDAPlace vs numeric
differences (the CPU twin is test_fluidk_cpu.py)."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import paddle_amd.fluid as fluid
from fluidk_cases import ACT_CASES, GRAD_CASES, rng
from op_test import OpTest
from paddle_amd.operators.math_ops import _ACT
from paddle_amd.ops import fluidk as fk

pytestmark = pytest.mark.gpu
dev = "cuda"


def _ab(name, attrs):
    keys = _ACT[name][1]
    if keys is None:
        return 0.0, 0.0
    d = dict(_ACT[name][0], **attrs)
    return float(d[keys[0]]) if keys[0] else 0.0, float(d[keys[1]]) if keys[1] else 0.0


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("name", sorted(ACT_CASES))
def test_activation_kernels_match_torch(name, dtype):
    attrs, lo, hi = ACT_CASES[name]
    a, b = _ab(name, attrs)
    _, _, fwd, dfn = _ACT[name]
    x32 = torch.empty(4099, device=dev).uniform_(lo, hi)  # odd size: vector body + tail
    x = x32.to(dtype)
    y = fk.act_fwd(name, x, a, b)
    ref = fwd(x.float(), a, b)
    tol = dict(atol=2e-5, rtol=2e-5) if dtype == torch.float32 else dict(atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(y.float(), ref, **tol)
    g = torch.randn(4099, device=dev).to(dtype)
    dx = fk.act_bwd(name, g, x, y, a, b)
    dref = g.float() * dfn(x.float(), y.float(), a, b)
    torch.testing.assert_close(dx.float(), dref, **(tol if dtype == torch.float32 else dict(atol=4e-2, rtol=4e-2)))


@pytest.mark.parametrize("V", [7, 1000, 32000])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_softmax_ce_kernel(V, dtype):
    x = (torch.randn(33, V, device=dev) * 3).to(dtype)
    lab = torch.randint(0, V, (33, 1), device=dev)
    lab[5] = -100
    prob, loss = fk.softmax_ce(x, lab, ignore_index=-100)
    lp = torch.log_softmax(x.float(), -1)
    ref = -lp.gather(1, lab.clamp_min(0))
    ref[5] = 0
    tol = dict(atol=1e-5, rtol=1e-5) if dtype == torch.float32 else dict(atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(prob.float(), lp.exp(), **tol)
    torch.testing.assert_close(loss.float(), ref, **tol)
    g = torch.rand(33, 1, device=dev)
    dx = fk.softmax_ce_grad(prob, g, lab, ignore_index=-100)
    oh = F.one_hot(lab.clamp_min(0).reshape(-1), V).float()
    dref = (lp.exp() - oh) * g
    dref[5] = 0
    torch.testing.assert_close(dx.float(), dref, **tol)
    soft = torch.softmax(torch.randn(33, V, device=dev), -1)
    prob, loss = fk.softmax_ce(x, soft=soft)
    torch.testing.assert_close(loss.float(), -(soft * lp).sum(-1, keepdim=True), **tol)
    dx = fk.softmax_ce_grad(prob, g, soft=soft)
    torch.testing.assert_close(dx.float(), (lp.exp() - soft) * g, **tol)


_DTS = [torch.float32, torch.bfloat16, torch.float16, torch.float64, torch.int32, torch.int64, torch.uint8,
        torch.bool, torch.int8, torch.int16]


@pytest.mark.parametrize("src", _DTS, ids=str)
def test_cast_kernel_matches_torch(src):
    x = (torch.randn(1031, device=dev, dtype=torch.float64) * 60)
    x[::7] = 0
    x = x.to(src)
    for dst in _DTS:
        y = fk.cast(x, dst)
        assert y.dtype == dst
        ref = x.to(dst)
        if dst.is_floating_point and src.is_floating_point:
            torch.testing.assert_close(y.double(), ref.double(), atol=0, rtol=0)
        elif dst == torch.bool:
            assert torch.equal(y, ref)
        elif not dst.is_floating_point and src.is_floating_point:
            # only the in-range values are defined behaviour for float -> narrow int
            info = torch.iinfo(dst)
            ok = (x.double() >= info.min) & (x.double() <= info.max)
            assert torch.equal(y[ok], ref[ok])
        else:
            assert torch.equal(y.double(), ref.double()), (src, dst)


def test_strided_gather_family():
    x = torch.randn(3, 4, 5, 6, device=dev)
    torch.testing.assert_close(fk.permute(x, [3, 1, 0, 2]), x.permute(3, 1, 0, 2).contiguous(), atol=0, rtol=0)
    torch.testing.assert_close(fk.flip(x, [0, 3]), torch.flip(x, [0, 3]), atol=0, rtol=0)
    torch.testing.assert_close(fk.slice_(x, [1, 3], [1, -4], [3, 100]), x[:, 1:3, :, 2:], atol=0, rtol=0)
    y = torch.randn(4, 1, 6, device=dev).to(torch.bfloat16)
    torch.testing.assert_close(fk.expand(y, [2, 4, 5, 6]), y.expand(2, 4, 5, 6), atol=0, rtol=0)
    torch.testing.assert_close(fk.tile(y, [2, 3, 1]), y.repeat(2, 3, 1), atol=0, rtol=0)
    with pytest.raises(IndexError):
        fk.gather(x, [10], [x.numel()])


def test_philox_random_stats_and_determinism():
    u = fk.random([1 << 20], "uniform", -2.0, 3.0, seed=1234)
    assert float(u.min()) >= -2.0 and float(u.max()) < 3.0
    assert abs(float(u.mean()) - 0.5) < 0.01
    assert abs(float(u.var()) - 25.0 / 12) < 0.02
    g = fk.random([1 << 20], "gaussian", 1.0, 2.0, seed=99)
    assert abs(float(g.mean()) - 1.0) < 0.01 and abs(float(g.std()) - 2.0) < 0.01
    assert torch.equal(fk.random([4097], "gaussian", 0, 1, seed=5), fk.random([4097], "gaussian", 0, 1, seed=5))
    assert not torch.equal(fk.random([4097], "uniform", 0, 1, seed=5), fk.random([4097], "uniform", 0, 1, seed=6))
    b = fk.random([3000], "uniform", 0, 1, seed=7, dtype=torch.bfloat16)
    assert b.dtype == torch.bfloat16 and 0 <= float(b.min()) and float(b.max()) <= 1


def test_random_ops_through_executor():
    prog, start = fluid.Program(), fluid.Program()
    with fluid.program_guard(prog, start):
        u = fluid.layers.uniform_random([512, 256], min=-1.0, max=1.0, seed=11)
        g = fluid.layers.gaussian_random([512, 256], mean=0.0, std=1.0, seed=0)
    exe = fluid.Executor(fluid.CUDAPlace(0))
    a, b = exe.run(prog, fetch_list=[u, g])
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == (512, 256) and -1 <= a.min() and a.max() < 1 and abs(a.mean()) < 0.02
    assert abs(b.std() - 1.0) < 0.02
    a2 = np.asarray(exe.run(prog, fetch_list=[u])[0])
    assert np.array_equal(a, a2)  # fixed op seed -> same stream


_LOSS_REF = {
    "hinge_loss": lambda x, y, a: (F.relu(1 - x * (2 * y - 1)), None),
    "huber_loss": lambda x, y, a: (torch.where((y - x).abs() <= a, 0.5 * (y - x) ** 2,
                                               a * ((y - x).abs() - 0.5 * a)), y - x),
    "log_loss": lambda x, y, a: (-y * torch.log(x + a) - (1 - y) * torch.log(1 - x + a), None),
    "modified_huber_loss": lambda x, y, a: (lambda z: (torch.where(z < -1, -4 * z, torch.where(
        z < 1, (1 - z) ** 2, torch.zeros_like(z))), z))(x * (2 * y - 1)),
    "sigmoid_cross_entropy_with_logits": lambda x, y, a: (
        F.binary_cross_entropy_with_logits(x, y, reduction="none"), None),
}


@pytest.mark.parametrize("name", sorted(_LOSS_REF))
def test_loss_kernels_match_torch(name):
    n = 5003
    if name == "log_loss":
        x = torch.rand(n, device=dev) * 0.8 + 0.1
        a = 1e-4
    else:
        x = torch.randn(n, device=dev) * 2
        a = 1.0
    y = (torch.rand(n, device=dev) > 0.5).float() if name != "huber_loss" else torch.randn(n, device=dev) * 2
    out, res = fk.loss_fwd(name, x, y, a, want_res=True)
    ref, rres = _LOSS_REF[name](x, y, a)
    torch.testing.assert_close(out, ref, atol=1e-5, rtol=1e-5)
    if rres is not None:
        torch.testing.assert_close(res, rres, atol=1e-6, rtol=1e-6)
    xr = x.clone().requires_grad_(True)
    g = torch.rand(n, device=dev)
    (_LOSS_REF[name](xr, y, a)[0] * g).sum().backward()
    dx = fk.loss_bwd(name, x, y, g, res=res, a=a)
    torch.testing.assert_close(dx, xr.grad, atol=1e-5, rtol=1e-4)


def test_seq_softmax_kernel():
    off = [0, 3, 3, 70, 1100, 1101]
    x = torch.randn(off[-1], device=dev) * 3
    y = fk.seq_softmax(x, off)
    ref = torch.cat([torch.softmax(x[s:e], 0) for s, e in zip(off[:-1], off[1:])])
    torch.testing.assert_close(y, ref, atol=1e-6, rtol=1e-5)
    g = torch.randn_like(x)
    dx = fk.seq_softmax_grad(y, g, off)
    dref = torch.cat([y[s:e] * (g[s:e] - (y[s:e] * g[s:e]).sum()) for s, e in zip(off[:-1], off[1:])])
    torch.testing.assert_close(dx, dref, atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("name", sorted(ACT_CASES))
def test_activation_grad_op_on_device(name):
    attrs, lo, hi = ACT_CASES[name]
    t = OpTest()
    t.op_type, t.inputs, t.attrs = name, {"X": rng.uniform(lo, hi, (3, 5)).astype("float32")}, attrs
    t.outputs = {"Out": np.zeros(1, "float32")}
    t.check_grad(["X"], ["Out"], max_relative_error=0.02, places=[fluid.CUDAPlace(0)])


@pytest.mark.parametrize("op,inputs,attrs,grad,out", GRAD_CASES, ids=[f"{c[0]}_{i}" for i, c in enumerate(GRAD_CASES)])
def test_explicit_grad_op_on_device(op, inputs, attrs, grad, out):
    t = OpTest()
    t.op_type, t.inputs, t.attrs = op, inputs, attrs
    t.outputs = {out: np.zeros(1, "float32")}
    t.check_grad(grad, [out], max_relative_error=0.02, places=[fluid.CUDAPlace(0)])


from fluidk_cases import SEQ_CASES  # noqa: E402


@pytest.mark.parametrize("op,inputs,attrs,grad,expect", SEQ_CASES, ids=[f"{c[0]}_{i}" for i, c in enumerate(SEQ_CASES)])
def test_sequence_ops_on_device(op, inputs, attrs, grad, expect):
    t = OpTest()
    t.op_type, t.inputs, t.attrs = op, inputs, attrs
    if expect is not None:
        t.outputs = {"Out": expect}
        t.check_output(atol=1e-4, rtol=1e-4, places=[fluid.CUDAPlace(0)])
    t.outputs = {"Out": np.zeros(1, "float32")}
    t.check_grad(grad, ["Out"], max_relative_error=0.02, places=[fluid.CUDAPlace(0)])
