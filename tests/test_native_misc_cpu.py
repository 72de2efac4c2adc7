"""ops_misc.hip on the C++ executor's host place vs the interpreter: every op (and its
gradient, where it has one) inside a small trained net, 3 SGD steps, losses to 1e-5,
no Python fallback."""
import numpy as np
import pytest
import torch

import paddle_amd.fluid as fluid
from paddle_amd.fluid.layers.layer_utils import simple_op
from paddle_amd.framework import core

from native_control_cases import run

L = fluid.layers


def _head(x):
    return L.fc(x, 6, bias_attr=False)


def case_clip(x, lab, idx):
    return L.mean(L.square(simple_op("clip", {"X": [_head(x)]}, {"min": -0.3, "max": 0.4})))


def case_clip_by_norm(x, lab, idx):
    return L.mean(simple_op("clip_by_norm", {"X": [_head(x)]}, {"max_norm": 0.5}))


def case_sign_minus(x, lab, idx):
    h = _head(x)
    m = simple_op("minus", {"X": [h], "Y": [L.scale(h, 0.3)]}, {})
    return L.mean(L.elementwise_mul(m, simple_op("sign", {"X": [h]}, {}, stop_gradient=True)))


def case_label_smooth(x, lab, idx):
    p = L.softmax(_head(x))
    return L.mean(L.square(simple_op("label_smooth", {"X": [p]}, {"epsilon": 0.2})))


def case_sigmoid_ce(x, lab, idx):
    h = _head(x)
    z = L.cast(L.greater_than(lab, L.fill_constant([1], "float32", 0.0)), "float32")
    return L.mean(simple_op("sigmoid_cross_entropy_with_logits", {"X": [h], "Label": [z]}, {"ignore_index": -100}))


def case_huber(x, lab, idx):
    h = _head(x)
    out, _ = simple_op("huber_loss", {"X": [h], "Y": [lab]}, {"delta": 0.5}, extra_outputs=("Residual",))
    return L.mean(out)


def case_log_loss(x, lab, idx):
    p = L.sigmoid(_head(x))
    z = L.cast(L.greater_than(lab, L.fill_constant([1], "float32", 0.0)), "float32")
    return L.mean(simple_op("log_loss", {"Predicted": [p], "Labels": [z]}, {"epsilon": 1e-4}, out_slot="Loss"))


def case_smooth_l1(x, lab, idx):
    h = _head(x)
    out, _ = simple_op("smooth_l1_loss", {"X": [h], "Y": [lab]}, {"sigma": 2.0}, extra_outputs=("Diff",))
    return L.mean(out)


def case_sq_l2(x, lab, idx):
    h = _head(x)
    d, _ = simple_op("squared_l2_distance", {"X": [h], "Y": [lab]}, {}, extra_outputs=("sub_result",))
    n = simple_op("squared_l2_norm", {"X": [h]}, {})
    return L.elementwise_add(L.mean(d), L.scale(n, 0.01))


def case_cumsum(x, lab, idx):
    h = _head(x)
    a = simple_op("cumsum", {"X": [h]}, {"axis": 1, "exclusive": True, "reverse": False})
    b = simple_op("cumsum", {"X": [h]}, {"axis": -1, "exclusive": False, "reverse": True})
    return L.mean(L.square(L.elementwise_add(a, b)))


def case_gather(x, lab, idx):
    h = _head(x)
    g = simple_op("gather", {"X": [h], "Index": [idx]}, {})
    return L.mean(L.square(g))


def case_one_hot_log_softmax(x, lab, idx):
    h = _head(x)
    oh = simple_op("one_hot", {"X": [idx]}, {"depth": 6, "dtype": 5}, stop_gradient=True)
    lsm = simple_op("log_softmax", {"X": [h]}, {"axis": -1})
    sel = simple_op("gather", {"X": [lsm], "Index": [idx]}, {})
    return L.elementwise_add(L.mean(L.elementwise_mul(oh, sel)), L.mean(L.square(lsm)))


def case_scatter(x, lab, idx):
    h = _head(x)
    up = L.scale(h, 2.0)
    s = simple_op("scatter", {"X": [h], "Ids": [idx], "Updates": [up]}, {"overwrite": False}, stop_gradient=True)
    return L.elementwise_add(L.mean(L.square(h)), L.mean(s))


CASES = {k[5:]: v for k, v in globals().items() if k.startswith("case_")}


def net(case):
    def build():
        x = L.data(name="x", shape=[5], dtype="float32")
        lab = L.data(name="lab", shape=[6], dtype="float32")
        idx = L.data(name="idx", shape=[1], dtype="int64")
        loss = CASES[case](x, lab, idx)
        fluid.optimizer.SGD(learning_rate=0.1).minimize(loss)
        return [loss]
    return build


def feeds(steps=3):
    out = []
    for s in range(steps):
        rs = np.random.RandomState(40 + s)
        out.append({"x": core.LoDTensor(torch.from_numpy(rs.randn(4, 5).astype("float32"))),
                    "lab": core.LoDTensor(torch.from_numpy(rs.randn(4, 6).astype("float32"))),
                    "idx": core.LoDTensor(torch.from_numpy(np.array([[2], [0], [3], [2]], dtype="int64")))})
    return out


@pytest.mark.parametrize("case", sorted(CASES))
def test_misc_op_native_host(case):
    fd = feeds()
    place = fluid.CPUPlace()
    ref, init, _ = run(net(case), fd, "python", place)
    got, _, exe = run(net(case), fd, "native", place, init)
    for a, b in zip(ref, got):
        np.testing.assert_allclose(b[0], a[0], rtol=1e-5, atol=1e-6)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks
