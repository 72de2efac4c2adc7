"""Parameter-server training (DistributeTranspiler + listen_and_serv over the native
TCP RPC) vs single-process training on the concatenated batch.

Reference test style: python/paddle/fluid/tests/unittests/test_dist_base.py
(pservers + trainers as local processes, losses compared with the local run) and
test_dist_transpiler.py (program structure after transpile).
"""
import multiprocessing as mp
import os
import traceback

import numpy as np
import pytest

from dist_util import _free_port

STEPS = 4


def _build(opt_name, distributed_table=False):
    import paddle_amd.fluid as fluid

    main, startup = fluid.Program(), fluid.Program()
    main.random_seed = startup.random_seed = 7
    with fluid.program_guard(main, startup):
        x = fluid.layers.data("x", shape=[16], dtype="float32")
        y = fluid.layers.data("y", shape=[1], dtype="float32")
        feats = [x]
        if distributed_table:
            ids = fluid.layers.data("ids", shape=[1], dtype="int64")
            emb = fluid.layers.embedding(ids, size=[50, 8], is_distributed=True, is_sparse=True,
                                         param_attr=fluid.ParamAttr(name="emb_table"))
            feats.append(fluid.layers.reshape(emb, [-1, 8]))
            x = fluid.layers.concat(feats, axis=1)
        h = fluid.layers.fc(x, 32, act="tanh")
        pred = fluid.layers.fc(h, 1)
        loss = fluid.layers.mean(fluid.layers.square_error_cost(pred, y))
        opt = {"sgd": lambda: fluid.optimizer.SGD(0.1),
               "momentum": lambda: fluid.optimizer.Momentum(0.05, momentum=0.9),
               "adam": lambda: fluid.optimizer.Adam(0.01),
               "adam_decay": lambda: fluid.optimizer.Adam(fluid.layers.exponential_decay(
                   0.01, decay_steps=2, decay_rate=0.5, staircase=True))}[opt_name]()
        opt.minimize(loss)
    return main, startup, loss


def _data(with_ids=False):
    rs = np.random.RandomState(3)
    X = rs.randn(STEPS, 16, 16).astype("float32")
    Y = rs.randn(STEPS, 16, 1).astype("float32")
    ids = rs.randint(0, 50, (STEPS, 16, 1)).astype("int64")
    return X, Y, ids


def _feed(i, lo, hi, with_ids):
    X, Y, ids = _data()
    f = {"x": X[i, lo:hi], "y": Y[i, lo:hi]}
    if with_ids:
        f["ids"] = ids[i, lo:hi]
    return f


def _local(opt_name, with_ids):
    import paddle_amd.fluid as fluid

    main, startup, loss = _build(opt_name, with_ids)
    exe = fluid.Executor(fluid.CPUPlace())
    scope = fluid.Scope()
    with fluid.scope_guard(scope):
        exe.run(startup)
        return [float(exe.run(main, feed=_feed(i, 0, 16, with_ids), fetch_list=[loss])[0].reshape(-1)[0]) for i in range(STEPS)]


def _worker(role, idx, eps, n_tr, opt_name, with_ids, q, sync=True):
    try:
        import paddle_amd.fluid as fluid

        main, startup, loss = _build(opt_name, with_ids)
        cfg = fluid.DistributeTranspilerConfig()
        cfg.min_block_size = 64  # force parameter slicing across both pservers
        t = fluid.DistributeTranspiler(cfg)
        t.transpile(idx if role == "trainer" else 0, program=main, pservers=",".join(eps), trainers=n_tr,
                    sync_mode=sync, startup_program=startup)
        exe = fluid.Executor(fluid.CPUPlace())
        scope = fluid.Scope()
        with fluid.scope_guard(scope):
            if role == "pserver":
                pmain, pstart = t.get_pserver_programs(eps[idx])
                exe.run(pstart)
                exe.run(pmain)
                q.put((role, idx, "ok"))
            else:
                tp = t.get_trainer_program()
                exe.run(startup)
                per = 16 // n_tr
                out = [float(exe.run(tp, feed=_feed(i, idx * per, (idx + 1) * per, with_ids),
                                     fetch_list=[loss])[0].reshape(-1)[0]) for i in range(STEPS)]
                exe.close()
                q.put((role, idx, out))
    except Exception:
        q.put((role, idx, "ERR " + traceback.format_exc()))


def _run_cluster(opt_name, with_ids=False, sync=True):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    eps = [f"127.0.0.1:{_free_port()}" for _ in range(2)]
    procs = [ctx.Process(target=_worker, args=("pserver", i, eps, 2, opt_name, with_ids, q, sync)) for i in range(2)]
    procs += [ctx.Process(target=_worker, args=("trainer", i, eps, 2, opt_name, with_ids, q, sync)) for i in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in procs:
            role, idx, r = q.get(timeout=240)
            assert not (isinstance(r, str) and r.startswith("ERR")), f"{role}{idx}: {r}"
            res[(role, idx)] = r
    finally:
        for p in procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
    return res


@pytest.mark.parametrize("opt_name", ["sgd", "momentum", "adam", "adam_decay"])
def test_pserver_sync_matches_local(opt_name):
    local = _local(opt_name, False)
    res = _run_cluster(opt_name)
    # mean of the two half-batch losses == full-batch loss (same params every step)
    dist = [(a + b) / 2 for a, b in zip(res[("trainer", 0)], res[("trainer", 1)])]
    np.testing.assert_allclose(dist, local, rtol=1e-4, atol=1e-5)
    assert local[-1] < local[0]


def test_transpiler_program_structure():
    import paddle_amd.fluid as fluid

    main, startup, loss = _build("momentum")
    cfg = fluid.DistributeTranspilerConfig()
    cfg.min_block_size = 64
    t = fluid.DistributeTranspiler(cfg)
    t.transpile(0, program=main, pservers="127.0.0.1:1,127.0.0.1:2", trainers=2, startup_program=startup)
    ops = [o.type for o in t.get_trainer_program().global_block().ops]
    assert "momentum" not in ops and "sgd" not in ops
    for o in ("split_byref", "send", "send_barrier", "recv", "fetch_barrier", "concat"):
        assert o in ops, o
    assert ops.index("send") < ops.index("send_barrier") < ops.index("recv") < ops.index("fetch_barrier")
    # the first fc weight is 16x32 = 512 elements -> 2 blocks, one per pserver
    w = next(p.name for p, _ in t.params_grads if list(p.shape) == [16, 32])
    names = [b[0] for b in t.blocks[w]]
    assert names == [w + ".block0", w + ".block1"]
    assert {b[3] for b in t.blocks[w]} == {"127.0.0.1:1", "127.0.0.1:2"}
    p0 = t.get_pserver_program("127.0.0.1:1")
    ls = p0.global_block().ops[-1]
    assert ls.type == "listen_and_serv" and ls.attrs["Fanin"] == 2
    sub = [o.type for b in ls.attrs["optimize_blocks"] for o in b.ops]
    assert "sum" in sub and "scale" in sub and "momentum" in sub
    # every trainer copy of a gradient routes to an optimize block
    assert all(":" in s and ".trainer_" in s for s in ls.attrs["grad_to_block_id"])


def test_pserver_distributed_lookup_table_matches_local():
    """embedding(is_distributed=True): rows sharded id % 2 over the pservers, fetched
    with prefetch, updated from SelectedRows gradients (SGD)."""
    local = _local("sgd", True)
    res = _run_cluster("sgd", with_ids=True)
    dist = [(a + b) / 2 for a, b in zip(res[("trainer", 0)], res[("trainer", 1)])]
    np.testing.assert_allclose(dist, local, rtol=1e-4, atol=1e-5)


def test_pserver_async_trains():
    res = _run_cluster("sgd", sync=False)
    for k in range(2):
        losses = res[("trainer", k)]
        assert all(np.isfinite(losses))


# ------------------------------------------------------------------ Trainer env roles
def _trainer_role_worker(env, q):
    try:
        os.environ.update(env)
        import paddle_amd.fluid as fluid

        def train_func():
            x = fluid.layers.data("x", shape=[16], dtype="float32")
            y = fluid.layers.data("y", shape=[1], dtype="float32")
            pred = fluid.layers.fc(fluid.layers.fc(x, 32, act="tanh"), 1)
            return fluid.layers.mean(fluid.layers.square_error_cost(pred, y))

        tr = fluid.Trainer(train_func, lambda: fluid.optimizer.SGD(0.1), place=fluid.CPUPlace())
        losses = []
        X, Y, _ = _data()
        idx, n_tr = int(env.get("PADDLE_TRAINER_ID", "0")), int(env.get("PADDLE_TRAINERS", "1"))
        per = 16 // n_tr

        def reader():  # the same batch every step: the loss must fall
            for _ in range(STEPS):
                yield list(zip(X[0, idx * per:(idx + 1) * per], Y[0, idx * per:(idx + 1) * per]))

        def handler(ev):
            if isinstance(ev, fluid.EndStepEvent):
                losses.append(float(np.asarray(ev.metrics[0]).reshape(-1)[0]))

        tr.train(1, handler, reader=reader, feed_order=["x", "y"])
        q.put((env["PADDLE_TRAINING_ROLE"], idx, losses if env["PADDLE_TRAINING_ROLE"] == "TRAINER" else "ok"))
    except Exception:
        q.put((env.get("PADDLE_TRAINING_ROLE"), env.get("PADDLE_TRAINER_ID"), "ERR " + traceback.format_exc()))


def test_trainer_transpiles_from_environment():
    """fluid.Trainer reads PADDLE_TRAINING_ROLE / PADDLE_PSERVER_IPS / ... and becomes a
    parameter server or a transpiled trainer (reference trainer.py:295-360)."""
    port = str(_free_port())
    base = {"PADDLE_PSERVER_IPS": "127.0.0.1", "PADDLE_PSERVER_PORT": port, "PADDLE_TRAINERS": "2",
            "PADDLE_CURRENT_IP": "127.0.0.1"}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    envs = [dict(base, PADDLE_TRAINING_ROLE="PSERVER", PADDLE_TRAINER_ID="0")]
    envs += [dict(base, PADDLE_TRAINING_ROLE="TRAINER", PADDLE_TRAINER_ID=str(i)) for i in range(2)]
    procs = [ctx.Process(target=_trainer_role_worker, args=(e, q)) for e in envs]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in procs:
            role, idx, r = q.get(timeout=240)
            assert not (isinstance(r, str) and r.startswith("ERR")), f"{role}{idx}: {r}"
            res[(role, idx)] = r
    finally:
        for p in procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
    a, b = res[("TRAINER", 0)], res[("TRAINER", 1)]
    assert len(a) == STEPS and len(b) == STEPS
    mean = [(u + v) / 2 for u, v in zip(a, b)]
    assert mean[-1] < mean[0]
