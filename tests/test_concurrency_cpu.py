"""CSP concurrency (reference tests/unittests/test_concurrency.py,
framework/channel_test.cc): unbuffered rendezvous between a Go block and the main
block, buffered channels, close semantics and Select."""
import threading

import numpy as np
import torch

import paddle_amd.fluid as fluid
from paddle_amd.framework import core
from paddle_amd.operators.concurrency_ops import Channel, join_go_threads


def test_channel_runtime_semantics():
    ch = Channel(capacity=2)
    assert ch.send(1) and ch.send(2)
    assert not ch.can_send()
    assert ch.recv() == (1, True)
    ch.close()
    assert ch.recv() == (2, True)          # drains after close
    assert ch.recv() == (None, False)
    assert ch.send(3) is False
    # unbuffered: a send completes only when a receiver takes it
    u = Channel(0)
    got = []
    t = threading.Thread(target=lambda: got.append(u.recv()))
    t.start()
    assert u.send("x") is True
    t.join(5)
    assert got == [("x", True)]


def _run(main, fetch, feed=None):
    exe = fluid.Executor(fluid.CPUPlace())
    with fluid.executor.scope_guard(core.Scope()):
        out = exe.run(main, feed=feed or {}, fetch_list=fetch)
    join_go_threads(5)
    return out


def test_go_send_main_recv():
    main, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, startup):
        x = fluid.layers.fill_constant(shape=[2, 3], dtype="float32", value=3.0)
        ch = fluid.make_channel(dtype="float32", capacity=0)
        with fluid.Go():
            y = fluid.layers.scale(x, scale=2.0)
            fluid.channel_send(ch, y)
        res = fluid.layers.fill_constant(shape=[2, 3], dtype="float32", value=0.0)
        out, status = fluid.channel_recv(ch, res)
        fluid.channel_close(ch)
    o, s = _run(main, [out, status])
    np.testing.assert_allclose(o, np.full((2, 3), 6.0, "float32"))
    assert bool(np.asarray(s).reshape(-1)[0])


def test_buffered_channel_producer_consumer():
    """Go block sends 5 values through a buffered channel; the main block sums them in a While."""
    main, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, startup):
        ch = fluid.make_channel(dtype="float32", capacity=5)
        with fluid.Go():
            for k in range(5):
                v = fluid.layers.fill_constant(shape=[1], dtype="float32", value=float(k + 1))
                fluid.channel_send(ch, v)
            fluid.channel_close(ch)
        acc = fluid.layers.fill_constant(shape=[1], dtype="float32", value=0.0)
        i = fluid.layers.fill_constant(shape=[1], dtype="int64", value=0)
        n = fluid.layers.fill_constant(shape=[1], dtype="int64", value=5)
        cond = fluid.layers.less_than(i, n)
        w = fluid.layers.While(cond)
        with w.block():
            tmp = fluid.layers.fill_constant(shape=[1], dtype="float32", value=0.0)
            got, _ = fluid.channel_recv(ch, tmp)
            fluid.layers.assign(fluid.layers.elementwise_add(acc, got), acc)
            fluid.layers.increment(i, in_place=True)
            fluid.layers.less_than(i, n, cond=cond)
    (a,) = _run(main, [acc])
    assert float(np.asarray(a).reshape(-1)[0]) == 15.0


def test_select_recv_and_default():
    main, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, startup):
        ch = fluid.make_channel(dtype="float32", capacity=1)
        one = fluid.layers.fill_constant(shape=[1], dtype="float32", value=7.0)
        fluid.channel_send(ch, one)
        result = fluid.layers.fill_constant(shape=[1], dtype="float32", value=-1.0)
        recv_into = fluid.layers.fill_constant(shape=[1], dtype="float32", value=0.0)
        with fluid.Select() as sel:
            with sel.case(fluid.channel_recv, ch, recv_into):
                fluid.layers.assign(fluid.layers.scale(recv_into, scale=10.0), result)
            with sel.default():
                fluid.layers.assign(fluid.layers.fill_constant(shape=[1], dtype="float32", value=99.0), result)
        # second select: channel now empty -> default case
        result2 = fluid.layers.fill_constant(shape=[1], dtype="float32", value=-1.0)
        with fluid.Select() as sel2:
            with sel2.case(fluid.channel_recv, ch, recv_into):
                fluid.layers.assign(recv_into, result2)
            with sel2.default():
                fluid.layers.assign(fluid.layers.fill_constant(shape=[1], dtype="float32", value=99.0), result2)
    r1, r2 = _run(main, [result, result2])
    assert float(np.asarray(r1).reshape(-1)[0]) == 70.0
    assert float(np.asarray(r2).reshape(-1)[0]) == 99.0
