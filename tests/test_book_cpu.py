"""Convergence ("book") tests (reference: python/paddle/fluid/tests/book/test_recognize_digits.py,
test_fit_a_line.py) and ParallelExecutor equivalence (parallel_executor_test_base.py:29,
test_parallel_executor_mnist.py:115-192: AllReduce vs Reduce strategies agree)."""
import os

import numpy as np
import pytest
import torch

import paddle_amd.fluid as fluid
from paddle_amd.framework import core


def _digits_data(n=512, seed=0):
    rng = np.random.RandomState(seed)
    X = rng.rand(n, 1, 28, 28).astype("float32")
    Y = X.reshape(n, -1)[:, :780].reshape(n, 10, 78).sum(-1).argmax(1).astype("int64").reshape(-1, 1)
    return X, Y


def mlp(img, label):
    hidden = fluid.layers.fc(input=img, size=64, act="tanh")
    hidden = fluid.layers.fc(input=hidden, size=64, act="tanh")
    prediction = fluid.layers.fc(input=hidden, size=10, act="softmax")
    loss = fluid.layers.cross_entropy(input=prediction, label=label)
    return prediction, fluid.layers.mean(loss), fluid.layers.accuracy(input=prediction, label=label)


def conv_net(img, label):
    c1 = fluid.nets.simple_img_conv_pool(input=img, filter_size=5, num_filters=20, pool_size=2, pool_stride=2,
                                         act="relu")
    c1 = fluid.layers.batch_norm(c1)
    c2 = fluid.nets.simple_img_conv_pool(input=c1, filter_size=5, num_filters=50, pool_size=2, pool_stride=2,
                                         act="relu")
    prediction = fluid.layers.fc(input=c2, size=10, act="softmax")
    loss = fluid.layers.cross_entropy(input=prediction, label=label)
    return prediction, fluid.layers.mean(loss), fluid.layers.accuracy(input=prediction, label=label)


def _train_digits(net, place, epochs=3, tmpdir=None):
    main, startup = fluid.Program(), fluid.Program()
    main.random_seed = startup.random_seed = 90
    with fluid.program_guard(main, startup):
        img = fluid.layers.data(name="img", shape=[1, 28, 28], dtype="float32")
        label = fluid.layers.data(name="label", shape=[1], dtype="int64")
        pred, loss, acc = net(img, label)
        test_prog = main.clone(for_test=True)
        fluid.optimizer.Adam(learning_rate=0.002).minimize(loss)
    exe = fluid.Executor(place)
    scope = core.Scope()
    X, Y = _digits_data()
    with fluid.executor.scope_guard(scope):
        exe.run(startup)
        first = None
        for ep in range(epochs):
            for i in range(0, len(X), 64):
                l, a = exe.run(main, feed={"img": X[i:i + 64], "label": Y[i:i + 64]}, fetch_list=[loss, acc])
                first = l if first is None else first
        tl, ta = exe.run(test_prog, feed={"img": X[:256], "label": Y[:256]}, fetch_list=[loss, acc])
        if tmpdir:
            fluid.io.save_inference_model(tmpdir, ["img"], [pred], exe, main_program=main)
            prog, feeds, fetches = fluid.io.load_inference_model(tmpdir, exe)
            (p1,) = exe.run(prog, feed={feeds[0]: X[:16]}, fetch_list=fetches)
            (p2,) = exe.run(test_prog, feed={"img": X[:16], "label": Y[:16]}, fetch_list=[pred])
            np.testing.assert_allclose(p1, p2, rtol=1e-4, atol=1e-5)
    return float(first[0]), float(tl[0]), float(ta[0])


def test_recognize_digits_mlp(tmp_path):
    first, last, acc = _train_digits(mlp, fluid.CPUPlace(), epochs=5, tmpdir=str(tmp_path / "mlp"))
    assert last < first and acc > 0.2


def test_recognize_digits_conv(tmp_path):
    first, last, acc = _train_digits(conv_net, fluid.CPUPlace(), epochs=3, tmpdir=str(tmp_path / "conv"))
    assert last < first and acc > 0.2


def test_fit_a_line():
    main, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, startup):
        x = fluid.layers.data(name="x", shape=[13], dtype="float32")
        y = fluid.layers.data(name="y", shape=[1], dtype="float32")
        y_predict = fluid.layers.fc(input=x, size=1, act=None)
        avg_cost = fluid.layers.mean(fluid.layers.square_error_cost(input=y_predict, label=y))
        fluid.optimizer.SGD(learning_rate=0.05).minimize(avg_cost)
    rng = np.random.RandomState(1)
    W = rng.rand(13, 1).astype("float32")
    X = rng.rand(256, 13).astype("float32")
    Yv = X @ W + 0.1
    exe = fluid.Executor(fluid.CPUPlace())
    scope = core.Scope()
    with fluid.executor.scope_guard(scope):
        exe.run(startup)
        for ep in range(60):
            for i in range(0, 256, 32):
                (l,) = exe.run(main, feed={"x": X[i:i + 32], "y": Yv[i:i + 32]}, fetch_list=[avg_cost])
    assert float(l[0]) < 0.05


def _pe_run(strategy, steps=4):
    main, startup = fluid.Program(), fluid.Program()
    main.random_seed = startup.random_seed = 7
    with fluid.program_guard(main, startup):
        img = fluid.layers.data(name="img", shape=[1, 28, 28], dtype="float32")
        label = fluid.layers.data(name="label", shape=[1], dtype="int64")
        _, loss, _ = mlp(img, label)
        fluid.optimizer.SGD(learning_rate=0.1).minimize(loss)
    scope = core.Scope()
    exe = fluid.Executor(fluid.CPUPlace())
    X, Y = _digits_data(256, 3)
    losses = []
    with fluid.executor.scope_guard(scope):
        exe.run(startup)
        if strategy is None:
            for i in range(steps):
                (l,) = exe.run(main, feed={"img": X[i * 32:(i + 1) * 32], "label": Y[i * 32:(i + 1) * 32]},
                               fetch_list=[loss])
                losses.append(float(l[0]))
        else:
            bs = fluid.BuildStrategy()
            bs.reduce_strategy = strategy
            pe = fluid.ParallelExecutor(use_cuda=False, loss_name=loss.name, main_program=main, build_strategy=bs,
                                        scope=scope)
            for i in range(steps):
                (l,) = pe.run([loss.name], feed={"img": X[i * 32:(i + 1) * 32], "label": Y[i * 32:(i + 1) * 32]})
                losses.append(float(np.mean(l)))
    return losses


def test_parallel_executor_allreduce_vs_reduce_vs_single(monkeypatch):
    monkeypatch.setenv("CPU_NUM", "2")
    single = _pe_run(None)
    ar = _pe_run(fluid.BuildStrategy.ReduceStrategy.AllReduce)
    rd = _pe_run(fluid.BuildStrategy.ReduceStrategy.Reduce)
    # first loss: same params, batch split in halves whose mean equals the full-batch mean
    assert abs(single[0] - ar[0]) < 1e-5
    for a, b in zip(ar, rd):
        assert abs(a - b) < 1e-5
    for a, b in zip(single, ar):
        assert abs(a - b) < 1e-4


def test_parallel_executor_ssa_graph_overlaps_allreduce(monkeypatch):
    """The step runs as one SSA graph on the native DAG pool: per-replica compute
    nodes, one all-reduce node per gradient bucket, optimizer nodes.  With
    one-gradient buckets the first bucket's all-reduce starts while the backward
    of earlier layers is still running (the trace of the step shows it)."""
    from paddle_amd.utils import flags as FLAGS

    monkeypatch.setenv("CPU_NUM", "2")
    old = FLAGS.get("rccl_bucket_mb")
    FLAGS.set("rccl_bucket_mb", 0)  # every gradient is its own bucket
    try:
        main, startup = fluid.Program(), fluid.Program()
        main.random_seed = startup.random_seed = 3
        with fluid.program_guard(main, startup):
            x = fluid.layers.data("x", [64])
            h = x
            for _ in range(6):
                h = fluid.layers.fc(h, 64, act="relu")
            loss = fluid.layers.mean(fluid.layers.fc(h, 1))
            fluid.optimizer.SGD(0.01).minimize(loss)
        scope = core.Scope()
        with fluid.executor.scope_guard(scope):
            fluid.Executor(fluid.CPUPlace()).run(startup)
            pe = fluid.ParallelExecutor(use_cuda=False, loss_name=loss.name, main_program=main, scope=scope,
                                        trace=True)
            pe.run([loss.name], feed={"x": np.random.rand(16, 64).astype("float32")})
        ev = pe.trace.events
        kinds = {e[0] for e in ev}
        assert {"compute", "allreduce", "optimize"} <= kinds
        n_ar = sum(1 for e in ev if e[0] == "allreduce")
        assert n_ar == 14  # 7 fc layers x (w, b)
        first_ar_start = min(e[3] for e in ev if e[0] == "allreduce")
        last_compute_end = max(e[4] for e in ev if e[0] == "compute")
        assert first_ar_start < last_compute_end, "all-reduce did not overlap the backward"
        # both replicas ran every forward/backward op
        assert {e[2] for e in ev if e[0] == "compute"} == {0, 1}
    finally:
        FLAGS.set("rccl_bucket_mb", old)


def _pe_mp_worker(rank, world):
    import os

    os.environ["CPU_NUM"] = "1"
    main, startup = fluid.Program(), fluid.Program()
    main.random_seed = startup.random_seed = 7
    with fluid.program_guard(main, startup):
        img = fluid.layers.data(name="img", shape=[1, 28, 28], dtype="float32")
        label = fluid.layers.data(name="label", shape=[1], dtype="int64")
        _, loss, _ = mlp(img, label)
        fluid.optimizer.SGD(learning_rate=0.1).minimize(loss)
    scope = core.Scope()
    X, Y = _digits_data(256, 3)
    out = []
    with fluid.executor.scope_guard(scope):
        fluid.Executor(fluid.CPUPlace()).run(startup)
        pe = fluid.ParallelExecutor(use_cuda=False, loss_name=loss.name, main_program=main, scope=scope)
        for i in range(4):
            lo = i * 32 + rank * 16
            (l,) = pe.run([loss.name], feed={"img": X[lo:lo + 16], "label": Y[lo:lo + 16]})
            out.append(float(np.mean(l)))
    return out


def test_parallel_executor_two_processes_matches_single():
    """One replica per process (gloo here, RCCL on the GPU): bucket all-reduce
    nodes across processes give the single-process full-batch trajectory."""
    from dist_util import run_dist

    single = _pe_run(None)
    res = run_dist(_pe_mp_worker, 2)
    for step in range(4):
        assert abs((res[0][step] + res[1][step]) / 2 - single[step]) < 1e-4, (res, single)


def test_memory_optimize_keeps_results():
    main, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, startup):
        x = fluid.layers.data("x", [8])
        h = fluid.layers.fc(fluid.layers.fc(x, 16, act="relu"), 4)
        loss = fluid.layers.mean(h)
        fluid.optimizer.SGD(0.1).minimize(loss)
    exe = fluid.Executor(fluid.CPUPlace())
    scope = core.Scope()
    xv = np.random.rand(4, 8).astype("float32")
    with fluid.executor.scope_guard(scope):
        exe.run(startup)
        (a,) = exe.run(main, feed={"x": xv}, fetch_list=[loss])
    fluid.memory_optimize(main)
    assert "delete_var" in [op.type for op in main.global_block().ops]


def test_memory_optimize_with_while_sub_block():
    """Control-flow aware liveness: parent-scope vars the loop body reads stay alive
    through the loop; body-local temporaries are released inside the body; the
    result is unchanged."""
    main, startup = fluid.Program(), fluid.Program()
    with fluid.program_guard(main, startup):
        x = fluid.layers.data("x", shape=[4], dtype="float32")
        scale = fluid.layers.scale(x, scale=2.0)          # read only inside the loop
        acc = fluid.layers.fill_constant([2, 4], "float32", 0.0)
        i = fluid.layers.fill_constant([1], "int64", 0)
        n = fluid.layers.fill_constant([1], "int64", 3)
        cond = fluid.layers.less_than(i, n)
        loop = fluid.layers.While(cond)
        with loop.block():
            t = fluid.layers.elementwise_mul(scale, scale)   # body-local temporary
            t2 = fluid.layers.scale(t, scale=0.5)
            fluid.layers.assign(fluid.layers.elementwise_add(acc, t2), acc)
            fluid.layers.increment(i, in_place=True)
            fluid.layers.less_than(i, n, cond=cond)
        out = fluid.layers.reduce_sum(acc)
    exe = fluid.Executor(fluid.CPUPlace())
    xv = np.arange(8, dtype="float32").reshape(2, 4)
    scope = core.Scope()
    with fluid.executor.scope_guard(scope):
        exe.run(startup)
        (ref,) = exe.run(main, feed={"x": xv}, fetch_list=[out])
        n_freed = fluid.memory_optimize(main, skip_opt_set=[out.name])  # fetch targets are kept by the caller
        assert n_freed and n_freed > 0
        gb = main.global_block()
        wi = [k for k, op in enumerate(gb.ops) if op.type == "while"][0]
        freed_before_loop = {nm for op in gb.ops[:wi] if op.type == "delete_var" for nm in op.input("X")}
        assert scale.name not in freed_before_loop  # still needed by the loop body
        body = main.block(1)
        assert any(op.type == "delete_var" for op in body.ops)
        (res,) = exe.run(main, feed={"x": xv}, fetch_list=[out])
    np.testing.assert_allclose(res, ref)
    np.testing.assert_allclose(res, [3 * 0.5 * float(((2 * xv) ** 2).sum())], rtol=1e-5)
