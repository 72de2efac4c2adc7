"""Fluid operators on the HIP device: the table-driven OpTest cases of
test_ops_cpu.py run through the Executor on CUDAPlace (reference:
unittests/op_test.py runs every place), analytic gradients of the native-kernel
ops on the device vs numeric differences, and the general op-library kernels
(csrc/kernels/oplib.hip) against plain PyTorch fp32 references."""
import numpy as np
import pytest
import torch

from op_test import OpTest
from test_ops_cpu import CASES
from test_ops_more_cpu import MORE

pytestmark = pytest.mark.gpu
dev = "cuda"


def _gpu_place():
    import paddle_amd.fluid as fluid

    return fluid.CUDAPlace(0)


@pytest.mark.parametrize("op,inputs,outputs,attrs,grad,grad_out,tol,atol,no_check", CASES,
                         ids=[f"{c[0]}_{i}" for i, c in enumerate(CASES)])
def test_op_on_device(op, inputs, outputs, attrs, grad, grad_out, tol, atol, no_check):
    t = OpTest()
    t.op_type, t.inputs, t.attrs = op, inputs, attrs
    t.outputs = {k: v for k, v in outputs.items() if v is not None}
    if t.outputs:
        t.check_output(atol=max(atol, 1e-4), rtol=1e-3, no_check_set=no_check, places=[_gpu_place()])
    else:
        t.outputs = {k: np.zeros(1, "float32") for k in outputs}
        t.check_output(exec_only=True, places=[_gpu_place()])


@pytest.mark.parametrize("op,inputs,outputs,attrs,grad,grad_out,tol,atol,no_check", MORE,
                         ids=[f"{c[0]}_{i}" for i, c in enumerate(MORE)])
def test_more_ops_on_device(op, inputs, outputs, attrs, grad, grad_out, tol, atol, no_check):
    t = OpTest()
    t.op_type, t.inputs, t.attrs = op, inputs, attrs
    t.outputs = {k: v for k, v in outputs.items() if v is not None}
    if t.outputs:
        t.check_output(atol=max(atol, 1e-4), rtol=1e-3, no_check_set=no_check, places=[_gpu_place()])
    else:
        t.outputs = {k: np.zeros(1, "float32") for k in outputs}
        t.check_output(exec_only=True, places=[_gpu_place()])


R_ = np.random.RandomState(7)


def _r(*s, lo=-1.0, hi=1.0):
    return R_.uniform(lo, hi, s).astype("float32")


GRAD_CASES = [
    ("elementwise_add", {"X": _r(3, 4, 5), "Y": _r(4, 1)}, {"axis": 1}, ["X", "Y"]),
    ("elementwise_mul", {"X": _r(3, 4, 5), "Y": _r(5)}, {}, ["X", "Y"]),
    ("elementwise_div", {"X": _r(3, 4), "Y": _r(3, 4, lo=0.5, hi=1.5)}, {}, ["X", "Y"]),
    ("elementwise_sub", {"X": _r(2, 3, 4), "Y": _r(3)}, {"axis": 1}, ["X", "Y"]),
    ("reduce_sum", {"X": _r(3, 4, 5)}, {"dim": [0, 2]}, ["X"]),
    ("reduce_mean", {"X": _r(3, 4, 5)}, {"dim": [1], "keep_dim": True}, ["X"]),
    # channel-first conv / pool on convnd.hip (vol2col + fp32 MFMA GEMM, gather pool backward)
    ("conv2d", {"Input": _r(2, 4, 6, 5), "Filter": _r(6, 2, 3, 3)},
     {"strides": [2, 1], "paddings": [1, 0], "dilations": [1, 2], "groups": 2}, ["Input", "Filter"]),
    ("conv3d", {"Input": _r(2, 3, 4, 5, 4), "Filter": _r(4, 3, 2, 3, 2)}, {"paddings": [1, 1, 0]},
     ["Input", "Filter"]),
    ("conv2d_transpose", {"Input": _r(2, 4, 3, 4), "Filter": _r(4, 3, 3, 3)},
     {"strides": [2, 2], "paddings": [1, 0]}, ["Input", "Filter"]),
    ("pool2d", {"X": _r(2, 3, 7, 6)}, {"pooling_type": "avg", "ksize": [3, 2], "strides": [2, 2],
                                       "paddings": [1, 1], "exclusive": True}, ["X"]),
    ("pool3d", {"X": _r(2, 2, 5, 4, 6)}, {"pooling_type": "avg", "ksize": [2, 2, 3], "strides": [2, 1, 2],
                                          "paddings": [1, 0, 1], "exclusive": False}, ["X"]),
]


@pytest.mark.parametrize("op,inputs,attrs,grad", GRAD_CASES, ids=[c[0] + str(i) for i, c in enumerate(GRAD_CASES)])
def test_native_op_grads_on_device(op, inputs, attrs, grad):
    t = OpTest()
    t.op_type, t.inputs, t.attrs = op, inputs, attrs
    out = "Output" if op.startswith("conv") else "Out"
    t.outputs = {out: np.zeros(1, "float32")}
    t.check_grad(grad, [out], max_relative_error=0.01, places=[_gpu_place()])


def test_sequence_pool_grad_on_device():
    x = _r(7, 3)
    for pt in ("SUM", "AVERAGE", "SQRT", "MAX", "LAST", "FIRST"):
        t = OpTest()
        t.op_type, t.inputs, t.attrs = "sequence_pool", {"X": (x, [[2, 5]])}, {"pooltype": pt}
        t.outputs = {"Out": np.zeros(1, "float32")}
        t.check_grad(["X"], ["Out"], max_relative_error=0.01, places=[_gpu_place()])


# ------------------------------------------------------------------ kernel level


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("op", ["add", "sub", "mul", "div", "max", "min", "pow"])
def test_binary_broadcast(op, dtype):
    from paddle_amd.ops import oplib

    g = torch.Generator(device=dev).manual_seed(1)
    x = (torch.rand(4, 3, 16, 8, generator=g, device=dev) + 0.5).to(dtype)
    for y in (torch.rand(4, 3, 16, 8, generator=g, device=dev) + 0.5, torch.rand(1, 3, 1, 8, generator=g, device=dev) + 0.5,
              torch.rand(1, 1, 1, 1, generator=g, device=dev) + 0.5):
        y = y.to(dtype)
        ref = {"add": torch.add, "sub": torch.sub, "mul": torch.mul, "div": torch.div, "max": torch.maximum,
               "min": torch.minimum, "pow": torch.pow}[op](x.float(), y.float())
        out = oplib.binary(op, x, y)
        assert _rel(out, ref) < (1e-6 if dtype == torch.float32 else 1e-2)


@pytest.mark.parametrize("op", ["sum", "mean", "max", "min", "prod"])
@pytest.mark.parametrize("dims", [[0], [1], [2], [0, 2], [1, 2], [0, 1, 2]])
def test_reduce(op, dims):
    from paddle_amd.ops import oplib

    g = torch.Generator(device=dev).manual_seed(2)
    x = torch.rand(5, 33, 70, generator=g, device=dev) + 0.5
    if op == "prod":
        x = 1 + (x - 0.5) * 1e-3  # keeps the product of 11550 terms in fp32 range
    out = oplib.reduce(op, x, dims, keep_dim=True)
    ref = {"sum": lambda t: t.sum(dims, keepdim=True), "mean": lambda t: t.mean(dims, keepdim=True),
           "max": lambda t: t.amax(dims, keepdim=True), "min": lambda t: t.amin(dims, keepdim=True),
           "prod": lambda t: t.double().prod(dims[0], keepdim=True) if len(dims) == 1 else
           t.double().log().sum(dims, keepdim=True).exp()}[op](x)
    assert out.shape == ref.shape
    assert _rel(out, ref) < 1e-4


def test_dropout_philox():
    from paddle_amd.ops import oplib

    x = torch.randn(1000, 257, device=dev)
    out, mask = oplib.dropout(x, 0.3, seed=1234, upscale=True)
    out2, mask2 = oplib.dropout(x, 0.3, seed=1234, upscale=True)
    keep = mask.float().mean().item()
    assert abs(keep - 0.7) < 0.01
    assert torch.allclose(out, x * mask.float() / 0.7, rtol=1e-6, atol=1e-6)
    assert not torch.equal(mask, mask2)  # the counter offset advances between calls
    g = torch.randn_like(x)
    assert torch.allclose(oplib.mask_mul(g, mask, 1 / 0.7), g * mask.float() / 0.7)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_topk(dtype):
    from paddle_amd.ops import oplib

    x = torch.randn(37, 1000, device=dev).to(dtype)
    v, i = oplib.topk(x, 16)
    rv, ri = torch.topk(x.float(), 16, -1)
    assert torch.equal(v.float(), rv)
    assert torch.equal(torch.gather(x.float(), 1, i), rv)


def test_sgd_adagrad_sparse():
    from paddle_amd.ops import oplib

    p, g = torch.randn(64, 32, device=dev), torch.randn(64, 32, device=dev)
    lr = torch.tensor([0.1], device=dev)
    ref = p - 0.1 * g
    assert torch.allclose(oplib.sgd_(p.clone(), g, lr), ref)
    m = torch.rand(64, 32, device=dev)
    pa = p.clone()
    ma = m.clone()
    oplib.adagrad_(pa, g, ma, lr, 1e-6)
    m2 = m + g * g
    assert torch.allclose(ma, m2) and torch.allclose(pa, p - 0.1 * g / (m2.sqrt() + 1e-6), atol=1e-6)
    rows = [3, 7, 3, 60]
    vals = torch.randn(4, 32, device=dev)
    ps = oplib.sgd_sparse_(p.clone(), rows, vals, lr)
    refs = p.clone().index_add_(0, torch.tensor(rows, device=dev), -0.1 * vals)
    assert torch.allclose(ps, refs, atol=1e-6)
    u, s = oplib.merge_rows(rows, vals)
    assert u == [3, 7, 60] and torch.allclose(s[0], vals[0] + vals[2])


def test_gather_scatter_rows():
    from paddle_amd.ops import oplib

    src = torch.randn(10, 6, device=dev, requires_grad=True)
    idx = [2, -1, 9, 2, 0]
    out = oplib.gather_rows_op(src, idx, 0.5)
    assert torch.equal(out[1], torch.full((6,), 0.5, device=dev))
    assert torch.equal(out[0], src[2]) and torch.equal(out[2], src[9])
    out.sum().backward()
    assert src.grad[2].eq(2).all() and src.grad[1].eq(0).all()


def test_gru_step_matches_reference():
    from paddle_amd.ops import oplib
    from paddle_amd.operators import rnn_ops

    g = torch.randn(5, 24, device=dev, requires_grad=True)
    h = torch.randn(5, 8, device=dev, requires_grad=True)
    W = torch.randn(8, 24, device=dev, requires_grad=True)
    outs = oplib.gru_step(g, h, W, 8)
    g2, h2, W2 = (t.detach().clone().requires_grad_() for t in (g, h, W))
    ur = g2[:, :16] + h2 @ W2[:, :16]
    u, r = torch.sigmoid(ur[:, :8]), torch.sigmoid(ur[:, 8:])
    rh = r * h2
    c = torch.tanh(g2[:, 16:] + rh @ W2[:, 16:])
    ref = (h2 - u * h2 + u * c, u, r, c, rh)
    for a, b in zip(outs, ref):
        assert torch.allclose(a, b, atol=1e-5)
    outs[0].sum().backward()
    ref[0].sum().backward()
    for a, b in ((g, g2), (h, h2), (W, W2)):
        assert torch.allclose(a.grad, b.grad, atol=1e-5)
    assert rnn_ops._gru_step  # the op path uses the same fused step
