"""Explicit Fluid grad kernels on CPUPlace: every activation's ``<name>_grad`` op
and the hand-written grads of transpose / expand / slice / reverse / cast / the
loss family / softmax_with_cross_entropy / sequence_softmax vs numeric central
differences (reference op_test.py:395 check_grad contract).  The same cases run
on the HIP kernels in test_fluidk_gpu.py."""
import numpy as np
import pytest

import paddle_amd.fluid as fluid
from fluidk_cases import ACT_CASES, GRAD_CASES, rng
from op_test import OpTest
from paddle_amd.framework import registry as R


@pytest.mark.parametrize("name", sorted(ACT_CASES))
def test_activation_grad_op_cpu(name):
    attrs, lo, hi = ACT_CASES[name]
    assert not R.is_auto_grad(name + "_grad"), "activation grads are explicit kernels"
    t = OpTest()
    t.op_type, t.inputs, t.attrs = name, {"X": rng.uniform(lo, hi, (3, 5)).astype("float32")}, attrs
    t.outputs = {"Out": np.zeros(1, "float32")}
    t.check_grad(["X"], ["Out"], max_relative_error=0.01, places=[fluid.CPUPlace()])


@pytest.mark.parametrize("op,inputs,attrs,grad,out", GRAD_CASES, ids=[f"{c[0]}_{i}" for i, c in enumerate(GRAD_CASES)])
def test_explicit_grad_op_cpu(op, inputs, attrs, grad, out):
    assert not R.is_auto_grad(op + "_grad")
    t = OpTest()
    t.op_type, t.inputs, t.attrs = op, inputs, attrs
    t.outputs = {out: np.zeros(1, "float32")}
    t.check_grad(grad, [out], max_relative_error=0.01, places=[fluid.CPUPlace()])


from fluidk_cases import SEQ_CASES  # noqa: E402


@pytest.mark.parametrize("op,inputs,attrs,grad,expect", SEQ_CASES, ids=[f"{c[0]}_{i}" for i, c in enumerate(SEQ_CASES)])
def test_sequence_ops_cpu(op, inputs, attrs, grad, expect):
    t = OpTest()
    t.op_type, t.inputs, t.attrs = op, inputs, attrs
    if expect is not None:
        t.outputs = {"Out": expect}
        t.check_output(atol=1e-5, places=[fluid.CPUPlace()])
    t.outputs = {"Out": np.zeros(1, "float32")}
    t.check_grad(grad, ["Out"], max_relative_error=0.01, places=[fluid.CPUPlace()])
