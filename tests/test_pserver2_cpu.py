"""Block-sharded parameter server of the legacy engine (distributed/pserver2.py,
reference paddle/legacy/pserver/ParameterServer2.cpp / ParameterClient2.cpp):
block layout, synchronous ADD_GRADIENT (all trainers' gradients averaged, one
optimizer step), ASYNC_SGD with lagged-gradient discard, AVERAGE_PARAMETER,
sparse-row GET, save / load, and v2 ``trainer.SGD(is_local=False)`` with two
trainer processes matching one local trainer on the whole batch."""
import multiprocessing as mp
import os
import sys
import threading

import numpy as np
import pytest

from paddle_amd.distributed import pserver2 as P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _servers(n, trainers):
    ss = [P.ParameterServer2(num_trainers=trainers).start() for _ in range(n)]
    return ss, ",".join(f"127.0.0.1:{s.port}" for s in ss)


def test_block_size_and_layout():
    assert P.calc_block_size([10], 2) == 1024  # floor 2^10
    assert P.calc_block_size([1 << 24], 1) == 1 << 18  # ~2^7 blocks per server
    ss, spec = _servers(3, 1)
    try:
        c = P.ParameterClient2(spec)
        rs = np.random.RandomState(0)
        params = {"w": rs.randn(300, 70).astype("float32"), "b": rs.randn(70).astype("float32")}
        got = c.init(params)
        for k in params:
            np.testing.assert_array_equal(got[k], params[k])
        # every block on exactly one server, the blocks spread over all three
        owned = [set(s.blocks) for s in ss]
        assert all(owned) and sum(len(o) for o in owned) == len(set().union(*owned))
        c.close()
    finally:
        for s in ss:
            s.stop()


def _trainer_thread(spec, tid, params, grads, out, opt_config, momentum=0.0):
    c = P.ParameterClient2(spec, trainer_id=tid)
    c.init(params, param_configs={k: {"momentum": momentum} for k in params}, opt_config=opt_config)
    for g in grads:
        out.append(c.add_gradient(g, num_samples=4))
    c.close()


@pytest.mark.parametrize("method", ["momentum", "adam"])
def test_sync_add_gradient_is_one_update_on_the_average(method):
    ss, spec = _servers(2, 2)
    try:
        rs = np.random.RandomState(1)
        params = {"w": rs.randn(50, 41).astype("float32"), "b": rs.randn(41).astype("float32")}
        steps = 3
        gs = [[{k: rs.randn(*v.shape).astype("float32") for k, v in params.items()} for _ in range(steps)]
              for _ in range(2)]
        oc = {"learning_method": method, "learning_rate": 0.1}
        mu = 0.9 if method == "momentum" else 0.0
        outs = [[], []]
        ts = [threading.Thread(target=_trainer_thread, args=(spec, t, params, gs[t], outs[t], oc, mu))
              for t in range(2)]
        ts[0].start()
        ts[1].start()
        for t in ts:
            t.join(60)
        # reference: the same rule on the averaged gradient, one step per batch
        ref = {k: v.astype(np.float64).copy() for k, v in params.items()}
        st = {k: [np.zeros_like(v), np.zeros_like(v)] for k, v in ref.items()}
        for i in range(steps):
            for k in ref:
                g = (gs[0][i][k].astype(np.float64) + gs[1][i][k]) / 2
                if method == "momentum":
                    st[k][0] = mu * st[k][0] - 0.1 * g
                    ref[k] += st[k][0]
                else:
                    t = i + 1
                    st[k][0] = 0.9 * st[k][0] + 0.1 * g
                    st[k][1] = 0.999 * st[k][1] + 0.001 * g * g
                    ref[k] -= 0.1 * np.sqrt(1 - 0.999 ** t) / (1 - 0.9 ** t) * st[k][0] / (np.sqrt(st[k][1]) + 1e-8)
            for t in range(2):
                for k in ref:
                    np.testing.assert_allclose(outs[t][i][k], ref[k], rtol=1e-5, atol=1e-5)
    finally:
        for s in ss:
            s.stop()


def test_async_sgd_discards_lagged_gradients_and_average_and_rows(tmp_path):
    ss, spec = _servers(2, 2)
    try:
        params = {"e": np.arange(40, dtype="float32").reshape(10, 4)}
        c0 = P.ParameterClient2(spec, trainer_id=0)
        c1 = P.ParameterClient2(spec, trainer_id=1)
        cfg = {"e": {"sparse_remote_update": True}}
        oc = {"learning_method": "momentum", "learning_rate": 1.0, "async_lagged_grad_discard_ratio": 1.0}
        t = threading.Thread(target=c1.init, args=(params, cfg, oc))
        t.start()
        c0.init(params, cfg, oc)
        t.join(30)
        assert c0.block_size["e"] == 4  # one row per block
        one = {"e": np.ones((10, 4), "float32")}
        c0.async_sgd(one)            # applied (lag 0)
        c0.async_sgd(one)            # applied (lag 0: trainer 0 saw the previous update)
        got = c1.async_sgd(one)      # trainer 1 is 2 updates behind >= 1.0 * 2 trainers: discarded
        np.testing.assert_allclose(got["e"], params["e"] - 2)
        assert sum(s.lagged_discarded for s in ss) > 0
        rows = c0.get_rows({"e": [1, 7]})
        np.testing.assert_allclose(rows["e"][7], params["e"][7] - 2)
        # model averaging over the two trainers
        a = {"e": np.full((10, 4), 2.0, "float32")}
        b = {"e": np.full((10, 4), 4.0, "float32")}
        res = [None]
        t = threading.Thread(target=lambda: res.__setitem__(0, c1.average_parameters(b)))
        t.start()
        r0 = c0.average_parameters(a)
        t.join(30)
        np.testing.assert_allclose(r0["e"], 3.0)
        np.testing.assert_allclose(res[0]["e"], 3.0)
        # per-server value vectors to disk and back
        c0.save_values(str(tmp_path))
        c0.send_parameter(P.SET_PARAM_ZERO, {"e": np.zeros((10, 4), "float32")})
        c0.load_values(str(tmp_path))
        np.testing.assert_allclose(c0.get_parameters()["e"], 3.0)
        c0.close()
        c1.close()
    finally:
        for s in ss:
            s.stop()


# ---------------------------------------------------------------- v2 remote training
def _v2_run(spec, tid, half, steps, q):
    sys.path.insert(0, ROOT)
    try:
        import paddle.v2 as paddle
        from paddle_amd import fluid

        fluid.default_startup_program().random_seed = 7
        paddle.init(use_gpu=False, trainer_count=1)
        import paddle_amd as pa

        pa.seed(7)
        x = paddle.layer.data(name="x", type=paddle.data_type.dense_vector(6))
        y = paddle.layer.data(name="y", type=paddle.data_type.dense_vector(1))
        h = paddle.layer.fc(input=x, size=5, act=paddle.activation.Tanh())
        pred = paddle.layer.fc(input=h, size=1, act=paddle.activation.Linear())
        cost = paddle.layer.square_error_cost(input=pred, label=y)
        params = paddle.parameters.create(cost)
        opt = paddle.optimizer.Momentum(momentum=0.5, learning_rate=0.05)
        kw = {} if spec is None else {"is_local": False, "pserver_spec": spec, "trainer_id": tid}
        tr = paddle.trainer.SGD(cost=cost, parameters=params, update_equation=opt, **kw)
        rs = np.random.RandomState(3)
        data = [(rs.randn(6).astype("float32"), rs.randn(1).astype("float32")) for _ in range(8 * steps)]
        batches = [data[i * 8:(i + 1) * 8] for i in range(steps)]
        if half is not None:
            batches = [b[half * 4:(half + 1) * 4] for b in batches]
        tr.train(reader=lambda: iter(batches), num_passes=1, feeding={"x": 0, "y": 1})
        q.put((tid, {k: np.array(params[k]) for k in params.keys()}, None))
    except Exception as e:
        import traceback

        q.put((tid, None, traceback.format_exc()[-3000:] + repr(e)))


def test_v2_remote_sgd_two_trainers_matches_local_full_batch():
    ss, spec = _servers(2, 2)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    try:
        ps = [ctx.Process(target=_v2_run, args=(spec, t, t, 4, q)) for t in range(2)]
        ps.append(ctx.Process(target=_v2_run, args=(None, 9, None, 4, q)))
        for p in ps:
            p.start()
        res = {}
        for _ in ps:
            tid, vals, err = q.get(timeout=300)
            assert err is None, err
            res[tid] = vals
        for p in ps:
            p.join(30)
    finally:
        for s in ss:
            s.stop()
    # names: the two trainer processes and the local one build the same program
    for k, v in res[9].items():
        np.testing.assert_allclose(res[0][k], v, rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(res[1][k], v, rtol=1e-4, atol=1e-5)
