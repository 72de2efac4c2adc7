"""The book programs of tests/test_book_cpu.py on the C++ executor
(``fluid.Executor(engine="native")``): from identical initial parameters the native
engine must follow the Python engine's trajectory (1e-5) -- MNIST MLP and conv +
batch-norm with Adam, fit-a-line with SGD, and a ``while`` sub-block program run by
Executor::RunWhile.  Reference: python/paddle/fluid/tests/book/test_recognize_digits.py,
test_fit_a_line.py; framework/executor.cc:125-353, operators/while_op.cc."""
import numpy as np
import pytest

import paddle_amd.fluid as fluid
from paddle_amd.framework import core

from test_book_cpu import _digits_data, conv_net, mlp


def _run(build, feeds, engine, place, init=None):
    main, startup = fluid.Program(), fluid.Program()
    main.random_seed = startup.random_seed = 90
    with fluid.unique_name.guard(), fluid.program_guard(main, startup):
        fetch = build()
    scope = core.Scope()
    out = []
    with fluid.executor.scope_guard(scope):
        fluid.Executor(place).run(startup)
        pers = [v.name for v in main.list_vars() if v.persistable and v.name not in ("feed", "fetch")
                and scope.find_var(v.name) is not None and scope.find_var(v.name).get() is not None]
        if init is None:
            init = {n: np.array(scope.find_var(n).get_tensor().numpy()) for n in pers}
        else:
            for n in pers:
                scope.find_var(n).get_tensor().set(init[n], place)
        exe = fluid.Executor(place, engine=engine)
        for fd in feeds:
            res = exe.run(main, feed=fd, fetch_list=fetch)
            out.append([np.array(r) for r in res])
    return out, init, exe


def _digits_feeds(steps=6):
    X, Y = _digits_data(256)
    return [{"img": X[i * 32:(i + 1) * 32], "label": Y[i * 32:(i + 1) * 32]} for i in range(steps)]


def _digits(net):
    def build():
        img = fluid.layers.data(name="img", shape=[1, 28, 28], dtype="float32")
        label = fluid.layers.data(name="label", shape=[1], dtype="int64")
        _, loss, acc = net(img, label)
        fluid.optimizer.Adam(learning_rate=0.002).minimize(loss)
        return [loss, acc]
    return build


def _fit_a_line():
    x = fluid.layers.data(name="x", shape=[13], dtype="float32")
    y = fluid.layers.data(name="y", shape=[1], dtype="float32")
    y_predict = fluid.layers.fc(input=x, size=1, act=None)
    avg_cost = fluid.layers.mean(fluid.layers.square_error_cost(input=y_predict, label=y))
    fluid.optimizer.SGD(learning_rate=0.05).minimize(avg_cost)
    return [avg_cost]


def _line_feeds(steps=8):
    rng = np.random.RandomState(1)
    W = rng.rand(13, 1).astype("float32")
    X = rng.rand(256, 13).astype("float32")
    Y = X @ W + 0.1
    return [{"x": X[i * 32:(i + 1) * 32], "y": Y[i * 32:(i + 1) * 32]} for i in range(steps)]


def _while_prog():
    x = fluid.layers.data("x", shape=[4], dtype="float32")
    scale = fluid.layers.scale(x, scale=2.0)
    acc = fluid.layers.fill_constant([2, 4], "float32", 0.0)
    i = fluid.layers.fill_constant([1], "int64", 0)
    n = fluid.layers.fill_constant([1], "int64", 3)
    cond = fluid.layers.less_than(i, n)
    loop = fluid.layers.While(cond)
    with loop.block():
        t = fluid.layers.elementwise_mul(scale, scale)
        fluid.layers.assign(fluid.layers.elementwise_add(acc, fluid.layers.scale(t, scale=0.5)), acc)
        fluid.layers.increment(i, in_place=True)
        fluid.layers.less_than(i, n, cond=cond)
    return [fluid.layers.reduce_sum(acc)]


CASES = {
    "mlp": (_digits(mlp), _digits_feeds),
    "conv_bn": (_digits(conv_net), lambda: _digits_feeds(4)),
    "fit_a_line": (_fit_a_line, _line_feeds),
    "while": (_while_prog, lambda: [{"x": np.arange(8, dtype="float32").reshape(2, 4)}] * 2),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_book_program_native_matches_python(case):
    build, feeds = CASES[case]
    fd = feeds()
    place = fluid.CPUPlace()
    ref, init, _ = _run(build, fd, "python", place)
    got, _, exe = _run(build, fd, "native", place, init=init)
    for r, g in zip(ref, got):
        for a, b in zip(r, g):
            np.testing.assert_allclose(b, a, rtol=1e-5, atol=1e-6)
    eng = exe._native
    assert not eng.py_fallbacks, eng.py_fallbacks  # every op ran on a C++ kernel
    if case == "while":
        np.testing.assert_allclose(got[0][0], [3 * 0.5 * float(((2 * np.arange(8.0)) ** 2).sum())], rtol=1e-5)
