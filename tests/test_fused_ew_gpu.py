"""fused_elemwise_activation kernel (fused_ew.hip) vs a plain fp32 torch composite:
every {add, mul} x {relu, scale} compound in both orders, same-shape and axis-
broadcast Y, forward, IntermediateOut and both gradients."""
import itertools

import pytest
import torch

from paddle_amd.ops import oplib

pytestmark = pytest.mark.gpu


def _ref(x, y, f0, f1, scale, axis):
    if y.shape != x.shape:
        ax = axis if axis >= 0 else x.dim() - y.dim()
        y = y.reshape((1,) * ax + tuple(y.shape) + (1,) * (x.dim() - ax - y.dim()))
    un = {"relu": torch.relu, "scale": lambda t: t * scale}
    bi = {"elementwise_add": torch.add, "elementwise_mul": torch.mul}
    if f0 in bi:
        inter = un[f1](y.expand_as(x) if y.shape != x.shape else y)
        return bi[f0](x, inter), inter
    inter = bi[f1](x, y)
    return un[f0](inter), inter


COMBOS = [(b, u) for b, u in itertools.product(["elementwise_add", "elementwise_mul"], ["relu", "scale"])]
COMBOS = COMBOS + [(u, b) for b, u in COMBOS]


@pytest.mark.parametrize("f0,f1", COMBOS)
@pytest.mark.parametrize("yshape,axis", [((6, 10, 12), -1), ((10,), 1), ((10, 12), 1), ((12,), -1)])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_fused_ew_act(f0, f1, yshape, axis, dt):
    g = torch.Generator().manual_seed(hash((f0, f1, yshape)) % 1000)
    x = torch.randn(6, 10, 12, generator=g).to(dt)
    y = torch.randn(*yshape, generator=g).to(dt)
    xr, yr = x.double().requires_grad_(True), y.double().requires_grad_(True)
    ref, inter_ref = _ref(xr, yr, f0, f1, 0.7, axis)
    xd, yd = x.cuda().requires_grad_(True), y.cuda().requires_grad_(True)
    out, inter = oplib.fused_ew_act(xd, yd, (f0, f1), axis, 0.7, True)
    tol = dict(rtol=1e-5, atol=1e-5) if dt == torch.float32 else dict(rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(out.double().cpu(), ref.detach(), **tol)
    torch.testing.assert_close(inter.double().cpu(), inter_ref.detach().expand_as(ref), **tol)
    gy = torch.randn(ref.shape, generator=g).to(dt)
    ref.backward(gy.double())
    out.backward(gy.cuda())
    torch.testing.assert_close(xd.grad.double().cpu(), xr.grad, **tol)
    tol_y = tol if dt == torch.float32 else dict(rtol=3e-2, atol=1e-1)
    torch.testing.assert_close(yd.grad.double().cpu(), yr.grad, **tol_y)


def test_fluid_op_routes_native():
    import numpy as np

    import paddle_amd.fluid as fluid
    from op_test import OpTest

    x = np.random.RandomState(0).randn(4, 5).astype("float32")
    y = np.random.RandomState(1).randn(5).astype("float32")
    t = OpTest()
    t.op_type, t.inputs = "fused_elemwise_activation", {"X": x, "Y": y}
    t.attrs = {"functor_list": ["relu", "elementwise_add"], "axis": 1}
    t.outputs = {"Out": np.maximum(x + y, 0)}
    t.check_output(places=[fluid.CUDAPlace(0)])
