"""DynamicRNN / While training (reference: tests/unittests/test_dyn_rnn.py,
test_while_op.py): forward over LoD sequences matches an independent PyTorch
recurrence, and while_grad's parameter/input gradients match autograd."""
import numpy as np
import torch

import paddle_amd.fluid as fluid
from paddle_amd.framework import core

D, H = 5, 6
LOD = [0, 3, 5, 9]


def _build():
    main, startup = fluid.Program(), fluid.Program()
    main.random_seed = startup.random_seed = 11
    with fluid.program_guard(main, startup):
        x = fluid.layers.data(name="x", shape=[D], dtype="float32", lod_level=1)
        x.stop_gradient = False
        drnn = fluid.layers.DynamicRNN()
        with drnn.block():
            word = drnn.step_input(x)
            prev = drnn.memory(shape=[H], value=0.0)
            hidden = fluid.layers.fc(input=[word, prev], size=H, act="tanh",
                                     param_attr=[fluid.ParamAttr(name="wx"), fluid.ParamAttr(name="wh")],
                                     bias_attr=fluid.ParamAttr(name="b"))
            drnn.update_memory(prev, hidden)
            drnn.output(hidden)
        out = drnn()
        loss = fluid.layers.mean(out * out)
        pg = fluid.backward.append_backward(loss)
    return main, startup, x, out, loss, pg


def _torch_ref(xv, wx, wh, b):
    outs = []
    for i in range(len(LOD) - 1):
        h = torch.zeros(H, dtype=torch.float64)
        for t in range(LOD[i], LOD[i + 1]):
            h = torch.tanh(xv[t] @ wx + h @ wh + b)
            outs.append(h)
    return torch.stack(outs)


def test_dynamic_rnn_forward_and_grads():
    main, startup, x, out, loss, pg = _build()
    assert any(op.type == "while_grad" for op in main.global_block().ops)
    exe = fluid.Executor(fluid.CPUPlace())
    scope = core.Scope()
    rng = np.random.RandomState(0)
    xv = rng.randn(LOD[-1], D).astype("float32")
    t = core.LoDTensor(torch.from_numpy(xv), [LOD])
    names = [g.name for _, g in pg]
    with fluid.executor.scope_guard(scope):
        exe.run(startup)
        res = exe.run(main, feed={"x": t}, fetch_list=[out, loss, "x@GRAD"] + names)
        params = {n: torch.from_numpy(np.array(scope.find_var(n).get().tensor.numpy())).double()
                  for n in ("wx", "wh", "b")}
    o, l, gx = res[0], res[1], res[2]
    grads = dict(zip([p.name for p, _ in pg], res[3:]))
    X = torch.from_numpy(xv).double().requires_grad_()
    P = {k: v.clone().requires_grad_() for k, v in params.items()}
    ref = _torch_ref(X, P["wx"], P["wh"], P["b"].reshape(-1))
    np.testing.assert_allclose(o, ref.detach().numpy(), rtol=1e-5, atol=1e-6)
    lr = (ref * ref).mean()
    lr.backward()
    np.testing.assert_allclose(float(np.asarray(l).reshape(-1)[0]), lr.item(), rtol=1e-5)
    np.testing.assert_allclose(gx, X.grad.numpy(), rtol=1e-4, atol=1e-6)
    for k in ("wx", "wh", "b"):
        np.testing.assert_allclose(np.asarray(grads[k]).reshape(P[k].shape), P[k].grad.numpy(), rtol=1e-4,
                                   atol=1e-6)


def test_dynamic_rnn_trains():
    main, startup = fluid.Program(), fluid.Program()
    main.random_seed = startup.random_seed = 3
    with fluid.program_guard(main, startup):
        x = fluid.layers.data(name="x", shape=[D], dtype="float32", lod_level=1)
        y = fluid.layers.data(name="y", shape=[1], dtype="float32", lod_level=1)
        drnn = fluid.layers.DynamicRNN()
        with drnn.block():
            word = drnn.step_input(x)
            prev = drnn.memory(shape=[H], value=0.0)
            hidden = fluid.layers.fc(input=[word, prev], size=H, act="tanh")
            drnn.update_memory(prev, hidden)
            drnn.output(hidden)
        pred = fluid.layers.fc(drnn(), size=1)
        loss = fluid.layers.mean(fluid.layers.square_error_cost(pred, y))
        fluid.optimizer.Adam(learning_rate=0.05).minimize(loss)
    exe = fluid.Executor(fluid.CPUPlace())
    rng = np.random.RandomState(1)
    xv = rng.randn(LOD[-1], D).astype("float32")
    yv = np.cumsum(xv[:, :1], 0).astype("float32") * 0.3
    with fluid.executor.scope_guard(core.Scope()):
        exe.run(startup)
        ls = [float(np.asarray(exe.run(main, feed={"x": core.LoDTensor(torch.from_numpy(xv), [LOD]),
                                                   "y": core.LoDTensor(torch.from_numpy(yv), [LOD])},
                                       fetch_list=[loss])[0]).reshape(-1)[0]) for _ in range(30)]
    assert ls[-1] < 0.5 * ls[0], ls


def test_dynamic_rnn_consecutive_batches_same_scope():
    """Batches of different length profiles run back to back in one scope (the
    reference's stacked_dynamic_lstm benchmark loop): tensor arrays and their
    gradients must not carry over from the previous run."""
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "benchmarks"))
    import reference_suite as rs

    main, startup, loss = rs.stacked_lstm_program(50, 8, 8)
    exe = fluid.Executor(fluid.CPUPlace())
    with fluid.executor.scope_guard(core.Scope()):
        exe.run(startup)
        for seed in range(3):
            lens = np.random.RandomState(seed).randint(1, 25, 6).tolist()
            off = np.concatenate([[0], np.cumsum(lens)]).tolist()
            ids = torch.randint(0, 50, (off[-1], 1))
            lab = torch.randint(0, 2, (len(lens), 1))
            (lv,) = exe.run(main, feed={"words": core.LoDTensor(ids, [off]), "label": core.LoDTensor(lab)},
                            fetch_list=[loss])
            assert np.isfinite(np.asarray(lv)).all()
