"""Reference operator types kept for ProgramDesc compatibility (operators/compat_ops.py):
recurrent (StaticRNN's op in the reference), parallel_do, read / create_custom_reader,
the op-level collectives, attention_lstm and the remaining conv/pool/fusion variants.
Each is checked against an independent PyTorch computation."""
import numpy as np
import torch

import paddle_amd.fluid as fluid
from paddle_amd.framework import core
from paddle_amd.fluid.framework import VarType


def _run(main, startup, feed, fetch, scope=None):
    exe = fluid.Executor(fluid.CPUPlace())
    scope = scope or core.Scope()
    with fluid.executor.scope_guard(scope):
        exe.run(startup)
        return exe.run(main, feed=feed, fetch_list=fetch), scope


def test_recurrent_op_forward_and_grad():
    T, B, D, H = 4, 3, 5, 6
    main, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, startup):
        gb = main.global_block()
        x = fluid.layers.data(name="x", shape=[T, B, D], dtype="float32", append_batch_size=False)
        x.stop_gradient = False
        h0 = fluid.layers.data(name="h0", shape=[B, H], dtype="float32", append_batch_size=False)
        w = fluid.layers.create_parameter([D, H], "float32", name="w")
        u = fluid.layers.create_parameter([H, H], "float32", name="u")
        sub = main.create_block()
        xt = sub.create_var(name="x", dtype="float32", shape=[B, D])
        hp = sub.create_var(name="h_prev", dtype="float32", shape=[B, H])
        a = sub.create_var(name="a", dtype="float32", shape=[B, H])
        b_ = sub.create_var(name="b", dtype="float32", shape=[B, H])
        s_ = sub.create_var(name="s", dtype="float32", shape=[B, H])
        h = sub.create_var(name="h", dtype="float32", shape=[B, H])
        sub.append_op(type="mul", inputs={"X": [xt], "Y": [w]}, outputs={"Out": [a]})
        sub.append_op(type="mul", inputs={"X": [hp], "Y": [u]}, outputs={"Out": [b_]})
        sub.append_op(type="elementwise_add", inputs={"X": [a], "Y": [b_]}, outputs={"Out": [s_]})
        sub.append_op(type="tanh", inputs={"X": [s_]}, outputs={"Out": [h]})
        main.rollback()
        out = gb.create_var(name="h", dtype="float32", shape=[T, B, H])
        scopes = gb.create_var(name="rnn_scopes", type=VarType.STEP_SCOPES)
        gb.append_op(type="recurrent", inputs={"inputs": [x], "initial_states": [h0], "parameters": [w, u]},
                     outputs={"outputs": [out], "step_scopes": [scopes]},
                     attrs={"ex_states": ["h_prev"], "states": ["h"], "sub_block": sub, "reverse": False})
        loss = fluid.layers.mean(out * out)
        fluid.backward.append_backward(loss)
    rng = np.random.RandomState(0)
    xv, hv = rng.randn(T, B, D).astype("float32"), rng.randn(B, H).astype("float32")
    (o, gx, gw), scope = _run(main, startup, {"x": xv, "h0": hv}, [out, "x@GRAD", "w@GRAD"])
    W = torch.from_numpy(np.array(scope.find_var("w").get().tensor)).requires_grad_()
    U = torch.from_numpy(np.array(scope.find_var("u").get().tensor))
    X = torch.from_numpy(xv).requires_grad_()
    hh, outs = torch.from_numpy(hv), []
    for t in range(T):
        hh = torch.tanh(X[t] @ W + hh @ U)
        outs.append(hh)
    ref = torch.stack(outs)
    np.testing.assert_allclose(o, ref.detach().numpy(), rtol=1e-5, atol=1e-6)
    (ref * ref).mean().backward()
    np.testing.assert_allclose(gx, X.grad.numpy(), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(gw, W.grad.numpy(), rtol=1e-4, atol=1e-6)


def test_parallel_do_splits_and_concats():
    main, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, startup):
        gb = main.global_block()
        x = fluid.layers.data(name="x", shape=[6, 4], dtype="float32", append_batch_size=False)
        sub = main.create_block()
        xi = sub.create_var(name="x", dtype="float32", shape=[-1, 4])
        y = sub.create_var(name="y", dtype="float32", shape=[-1, 4])
        sub.append_op(type="scale", inputs={"X": [xi]}, outputs={"Out": [y]}, attrs={"scale": 2.0})
        main.rollback()
        out = gb.create_var(name="y", dtype="float32", shape=[6, 4])
        places = gb.create_var(name="places", dtype="float32")
        gb.append_op(type="get_places", inputs={}, outputs={"Out": [places]}, attrs={"device_count": 3})
        gb.append_op(type="parallel_do", inputs={"inputs": [x], "parameters": [], "places": [places]},
                     outputs={"outputs": [out]}, attrs={"sub_block": sub})
    xv = np.arange(24, dtype="float32").reshape(6, 4)
    (o,), _ = _run(main, startup, {"x": xv}, [out])
    np.testing.assert_allclose(o, 2 * xv)


def test_read_and_custom_reader_ops():
    class R:
        def __init__(self):
            self.i = 0

        def next_feed(self):
            self.i += 1
            return [core.LoDTensor(torch.full((2, 3), float(self.i)))]

    main, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, startup):
        gb = main.global_block()
        rd = gb.create_var(name="reader", type=VarType.READER)
        sub = main.create_block()
        src = sub.create_var(name="src", dtype="float32", shape=[2, 3])
        snk = sub.create_var(name="snk", dtype="float32", shape=[2, 3])
        sub.append_op(type="scale", inputs={"X": [src]}, outputs={"Out": [snk]}, attrs={"scale": 10.0})
        main.rollback()
        crd = gb.create_var(name="custom", type=VarType.READER)
        gb.append_op(type="create_custom_reader", inputs={"UnderlyingReader": [rd]}, outputs={"Out": [crd]},
                     attrs={"sub_block": sub, "source_var_names": ["src"], "sink_var_names": ["snk"]})
        out = gb.create_var(name="batch", dtype="float32", shape=[2, 3])
        gb.append_op(type="read", inputs={"Reader": [crd]}, outputs={"Out": [out]})
    exe = fluid.Executor(fluid.CPUPlace())
    scope = core.Scope()
    with fluid.executor.scope_guard(scope):
        scope.var("reader").set(R())
        exe.run(startup)
        (o1,) = exe.run(main, fetch_list=[out])
        (o2,) = exe.run(main, fetch_list=[out])
    assert float(np.asarray(o1)[0, 0]) == 10.0 and float(np.asarray(o2)[0, 0]) == 20.0


def test_single_process_collective_ops_are_identity():
    main, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, startup):
        gb = main.global_block()
        x = fluid.layers.data(name="x", shape=[3], dtype="float32", append_batch_size=False)
        comm = gb.create_var(name="comm", type=VarType.RAW)
        gb.append_op(type="ncclInit", inputs={}, outputs={"Communicator": [comm]})
        outs = []
        for t in ("ncclAllReduce", "ncclReduce", "ncclBcast"):
            o = gb.create_var(name=f"o_{t}", dtype="float32", shape=[3])
            gb.append_op(type=t, inputs={"X": [x], "Communicator": [comm]}, outputs={"Out": [o]})
            outs.append(o)
    xv = np.array([1.0, 2.0, 3.0], dtype="float32")
    res, _ = _run(main, startup, {"x": xv}, outs)
    for r in res:
        np.testing.assert_allclose(r, xv)


def _op_program(build):
    main, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, startup):
        fetch = build(main.global_block())
    return main, startup, fetch


def test_depthwise_conv2d_transpose_and_maxpool3d_index():
    C = 4
    x = np.random.RandomState(1).randn(2, C, 5, 5).astype("float32")
    w = np.random.RandomState(2).randn(C, 1, 3, 3).astype("float32")
    v = np.random.RandomState(3).randn(1, 2, 4, 4, 4).astype("float32")

    def build(gb):
        xi = fluid.layers.data(name="x", shape=list(x.shape), dtype="float32", append_batch_size=False)
        wi = fluid.layers.data(name="w", shape=list(w.shape), dtype="float32", append_batch_size=False)
        vi = fluid.layers.data(name="v", shape=list(v.shape), dtype="float32", append_batch_size=False)
        o = gb.create_var(name="o", dtype="float32")
        gb.append_op(type="depthwise_conv2d_transpose", inputs={"Input": [xi], "Filter": [wi]},
                     outputs={"Output": [o]}, attrs={"strides": [2, 2], "paddings": [1, 1], "groups": C})
        p = gb.create_var(name="p", dtype="float32")
        m = gb.create_var(name="m", dtype="int32")
        gb.append_op(type="max_pool3d_with_index", inputs={"X": [vi]}, outputs={"Out": [p], "Mask": [m]},
                     attrs={"ksize": [2, 2, 2], "strides": [2, 2, 2]})
        return [o, p, m]

    main, startup, fetch = _op_program(build)
    (o, p, m), _ = _run(main, startup, {"x": x, "w": w, "v": v}, fetch)
    ref = torch.nn.functional.conv_transpose2d(torch.from_numpy(x), torch.from_numpy(w), stride=2, padding=1,
                                               groups=C)
    np.testing.assert_allclose(o, ref.numpy(), rtol=1e-5, atol=1e-5)
    rp, ri = torch.nn.functional.max_pool3d(torch.from_numpy(v), 2, 2, return_indices=True)
    np.testing.assert_allclose(p, rp.numpy())
    np.testing.assert_array_equal(np.asarray(m), ri.numpy())


def test_fusion_seqexpand_concat_fc():
    lod = [0, 2, 5]
    x0 = np.random.RandomState(0).randn(5, 3).astype("float32")
    x1 = np.random.RandomState(1).randn(2, 2).astype("float32")
    W = np.random.RandomState(2).randn(5, 4).astype("float32")
    bb = np.random.RandomState(3).randn(4).astype("float32")

    def build(gb):
        a = fluid.layers.data(name="a", shape=[3], dtype="float32", lod_level=1)
        b = fluid.layers.data(name="b", shape=[2], dtype="float32")
        w = fluid.layers.data(name="w", shape=[5, 4], dtype="float32", append_batch_size=False)
        bias = fluid.layers.data(name="bias", shape=[4], dtype="float32", append_batch_size=False)
        o = gb.create_var(name="o", dtype="float32")
        f = gb.create_var(name="f", dtype="float32")
        gb.append_op(type="fusion_seqexpand_concat_fc", inputs={"X": [a, b], "FCWeight": [w], "FCBias": [bias]},
                     outputs={"Out": [o], "FCOut": [f]}, attrs={"fc_activation": "relu"})
        return [o]

    main, startup, fetch = _op_program(build)
    (o,), _ = _run(main, startup, {"a": core.LoDTensor(torch.from_numpy(x0), [lod]), "b": x1, "w": W,
                                   "bias": bb}, fetch)
    rep = np.repeat(x1, [2, 3], axis=0)
    ref = np.maximum(np.concatenate([x0, rep], 1) @ W + bb, 0)
    np.testing.assert_allclose(o, ref, rtol=1e-5, atol=1e-5)


def test_attention_lstm_matches_stepwise_reference():
    lod = [0, 3, 4]
    M, D = 3, 2
    rng = np.random.RandomState(0)
    X = rng.randn(4, M).astype("float32")
    C0 = rng.randn(2, D).astype("float32")
    AW = rng.randn(M + D, 1).astype("float32")
    LW = rng.randn(D + M, 4 * D).astype("float32")
    LB = rng.randn(1, 4 * D).astype("float32")

    def build(gb):
        names = {}
        for n, arr, lvl in (("X", X, 1), ("C0", C0, 0), ("AW", AW, 0), ("LW", LW, 0), ("LB", LB, 0)):
            names[n] = fluid.layers.data(name=n, shape=list(arr.shape[1:]) if lvl else list(arr.shape),
                                         dtype="float32", lod_level=lvl, append_batch_size=bool(lvl))
        outs = {k: gb.create_var(name=k.lower(), dtype="float32") for k in
                ("Hidden", "Cell", "AttentionedX", "AttentionFCOut", "LSTMX", "LSTMOUT")}
        gb.append_op(type="attention_lstm", inputs={"X": [names["X"]], "C0": [names["C0"]],
                                                    "AttentionWeight": [names["AW"]], "LSTMWeight": [names["LW"]],
                                                    "LSTMBias": [names["LB"]]},
                     outputs={k: [v] for k, v in outs.items()})
        return [outs["Hidden"], outs["Cell"]]

    main, startup, fetch = _op_program(build)
    (h, c), _ = _run(main, startup, {"X": core.LoDTensor(torch.from_numpy(X), [lod]), "C0": C0, "AW": AW,
                                     "LW": LW, "LB": LB}, fetch)
    sig = lambda v: 1 / (1 + np.exp(-v))  # noqa: E731
    H, Cc = np.zeros((4, D), "float32"), np.zeros((4, D), "float32")
    for i in range(2):
        xs = X[lod[i]:lod[i + 1]]
        cp, hp = C0[i], None
        for t in range(len(xs)):
            fc = np.maximum(xs @ AW[:M, 0] + cp @ AW[M:, 0], 0)
            a = np.exp(fc - fc.max())
            a /= a.sum()
            lx = a @ xs
            g = lx @ LW[D:] + (hp @ LW[:D] if hp is not None else 0) + LB[0]
            f, ig, o = sig(g[:D]), sig(g[D:2 * D]), sig(g[2 * D:3 * D])
            cp = f * cp + ig * np.tanh(g[3 * D:])
            hp = np.tanh(cp) * o
            H[lod[i] + t], Cc[lod[i] + t] = hp, cp
    np.testing.assert_allclose(h, H, rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(c, Cc, rtol=1e-4, atol=1e-5)
