"""The optimizer OpTest table (test_optimizer_ops_cpu.py) on CUDAPlace: dense fp32
updates run the fused kernels of optimizer.hip / optim_ext.hip."""
import pytest

import paddle_amd.fluid as fluid
from test_optimizer_ops_cpu import OPT_CASES, run_case

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("op,inputs,outputs,attrs", OPT_CASES, ids=[f"{c[0]}_{i}" for i, c in enumerate(OPT_CASES)])
def test_optimizer_op_on_device(op, inputs, outputs, attrs):
    run_case(op, inputs, outputs, attrs, fluid.CUDAPlace(0))


def test_native_kernels_are_used(monkeypatch):
    from paddle_amd.ops import oplib

    calls = []
    orig = oplib.opt_update_

    def spy(kind, *a, **k):
        r = orig(kind, *a, **k)
        calls.append((kind, r is not None))
        return r

    monkeypatch.setattr(oplib, "opt_update_", spy)
    for op, inputs, outputs, attrs in OPT_CASES:
        if op in ("adamax", "ftrl", "rmsprop", "lars_momentum", "adadelta", "decayed_adagrad", "proximal_gd"):
            run_case(op, inputs, outputs, attrs, fluid.CUDAPlace(0))
    assert calls and all(ok for _, ok in calls), calls
