"""Every activation of the op library, forward and backward, on the C++ executor's
host kernels (csrc/native/ops_host.cc) vs the interpreter: an fc feeding the
activation, trained for 3 SGD steps; losses and the trained weight agree to 1e-5 and
nothing falls back to a Python kernel."""
import numpy as np
import pytest
import torch

import paddle_amd.fluid as fluid
from paddle_amd.fluid.layers.nn import simple_op
from paddle_amd.framework import core

from native_control_cases import run

ACTS = {
    "relu": {}, "sigmoid": {}, "logsigmoid": {}, "exp": {}, "tanh": {}, "tanh_shrink": {},
    "softshrink": {"lambda": 0.3}, "sqrt": {}, "rsqrt": {}, "abs": {}, "ceil": {}, "floor": {}, "cos": {},
    "sin": {}, "round": {}, "reciprocal": {}, "log": {}, "square": {}, "softplus": {}, "softsign": {},
    "brelu": {"t_min": 0.1, "t_max": 1.5}, "leaky_relu": {"alpha": 0.1}, "soft_relu": {"threshold": 2.0},
    "elu": {"alpha": 0.7}, "relu6": {"threshold": 1.2}, "pow": {"factor": 2.5}, "stanh": {"scale_a": 0.5, "scale_b": 1.3},
    "hard_shrink": {"threshold": 0.4}, "thresholded_relu": {"threshold": 0.3},
    "hard_sigmoid": {"slope": 0.3, "offset": 0.4}, "swish": {"beta": 1.3}, "gelu": {}, "silu": {},
}
POSITIVE = {"sqrt", "rsqrt", "log", "reciprocal", "pow"}  # domain x > 0


def net(act, attrs):
    def build():
        x = fluid.layers.data(name="x", shape=[6], dtype="float32")
        h = fluid.layers.fc(x, 5, bias_attr=False)
        if act in POSITIVE:
            h = fluid.layers.elementwise_add(fluid.layers.square(h), fluid.layers.fill_constant([1], "float32", 0.5))
        y = simple_op(act, {"X": [h]}, dict(attrs))
        loss = fluid.layers.mean(fluid.layers.square(y))
        fluid.optimizer.SGD(learning_rate=0.05).minimize(loss)
        return [loss]
    return build


def feeds(steps=3):
    rs = np.random.RandomState(5)
    return [{"x": core.LoDTensor(torch.from_numpy(rs.randn(4, 6).astype("float32")))} for _ in range(steps)]


@pytest.mark.parametrize("act", sorted(ACTS))
def test_activation_native_host(act):
    fd = feeds()
    place = fluid.CPUPlace()
    ref, init, _ = run(net(act, ACTS[act]), fd, "python", place)
    got, _, exe = run(net(act, ACTS[act]), fd, "native", place, init)
    for a, b in zip(ref, got):
        np.testing.assert_allclose(b[0], a[0], rtol=1e-5, atol=1e-6)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks
