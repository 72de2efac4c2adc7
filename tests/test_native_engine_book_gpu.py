"""The book programs on the C++ executor with a HIP place: device kernels
(ops_gpu.hip) on torch's current stream, host kernels for the rest, and the
while sub-block run by Executor::RunWhile -- the trajectory must match the Python
engine on the same device."""
import numpy as np
import pytest

import paddle_amd.fluid as fluid

from test_native_engine_book_cpu import CASES, _run

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", sorted(CASES))
def test_book_program_native_matches_python_gpu(case):
    build, feeds = CASES[case]
    fd = feeds()
    place = fluid.CUDAPlace(0)
    ref, init, _ = _run(build, fd, "python", place)
    got, _, exe = _run(build, fd, "native", place, init=init)
    for r, g in zip(ref, got):
        for a, b in zip(r, g):
            np.testing.assert_allclose(b, a, rtol=2e-4, atol=2e-5)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks
    # every op ran on a device kernel: no host copy-in / copy-out round trips
    assert not exe._native.host_fallbacks(), exe._native.host_fallbacks()


def _tiny_transformer():
    """lookup_table -> fc -> layer_norm -> fc -> softmax / cross_entropy + top_k /
    accuracy with Adam: the device kernels of layer_norm(_grad), lookup_table_grad,
    top_k and accuracy (ops_gpu.hip) must reproduce the Python engine."""
    ids = fluid.layers.data(name="ids", shape=[1], dtype="int64")
    label = fluid.layers.data(name="label", shape=[1], dtype="int64")
    emb = fluid.layers.embedding(ids, size=[50, 32])
    h = fluid.layers.fc(emb, size=64, act="relu")
    h = fluid.layers.layer_norm(h, begin_norm_axis=1)
    pred = fluid.layers.fc(h, size=10, act="softmax")
    loss = fluid.layers.mean(fluid.layers.cross_entropy(pred, label))
    acc = fluid.layers.accuracy(input=pred, label=label, k=3)
    fluid.optimizer.Adam(learning_rate=0.01).minimize(loss)
    return [loss, acc]


def _tt_feeds(steps=6):
    rs = np.random.RandomState(7)
    out = []
    for _ in range(steps):
        i = rs.randint(0, 50, size=(32, 1)).astype("int64")
        out.append({"ids": i, "label": (i % 10).astype("int64")})
    return out


def test_transformer_ops_native_matches_python_gpu():
    place = fluid.CUDAPlace(0)
    fd = _tt_feeds()
    ref, init, _ = _run(_tiny_transformer, fd, "python", place)
    got, _, exe = _run(_tiny_transformer, fd, "native", place, init=init)
    for r, g in zip(ref, got):
        for a, b in zip(r, g):
            np.testing.assert_allclose(b, a, rtol=2e-4, atol=2e-5)
    fb = exe._native.py_fallbacks
    for op in ("layer_norm", "layer_norm_grad", "lookup_table_grad", "top_k", "accuracy"):
        assert op not in fb, fb
    assert not exe._native.host_fallbacks(), exe._native.host_fallbacks()
