"""Elastic parameter server (reference go/pserver: service_test.go, client_test.go,
etcd_client_test.go): slot registration with leases, FNV partitioning, optimizer
updates on the server, periodic CRC-checked checkpoints and resume after a
restart."""
import os
import time

import numpy as np
import pytest

from paddle_amd.distributed import pserver as ps


@pytest.fixture
def store(tmp_path):
    return ps.KVStore(str(tmp_path / "kv.json"))


def test_registration_leases(store):
    r0 = ps.register_pserver(store, 2, "127.0.0.1:1", ttl=0.6)
    r1 = ps.register_pserver(store, 2, "127.0.0.1:2", ttl=0.6)
    assert (r0.index, r1.index) == (0, 1)
    with pytest.raises(TimeoutError):
        ps.register_pserver(store, 2, "127.0.0.1:3", ttl=0.6, timeout=0.3)
    time.sleep(0.8)  # keep-alive threads refresh the leases
    assert ps.list_pservers(store) == [(0, "127.0.0.1:1"), (1, "127.0.0.1:2")]
    r1.close(release=False)  # a crashed server: its lease runs out
    time.sleep(0.9)
    assert ps.list_pservers(store) == [(0, "127.0.0.1:1")]
    r2 = ps.register_pserver(store, 2, "127.0.0.1:4", ttl=0.6)
    assert r2.index == 1
    r0.close()
    r2.close()


def test_fnv_partition_matches_go():
    assert ps.fnv1a32("") == 0x811C9DC5
    assert ps.fnv1a32("a") == 0xE40C292C  # FNV-1a 32 test vector


def _servers(store, tmp_path, n=2, interval=0.0):
    return [ps.PServer(store, n, str(tmp_path / "ckpt"), checkpoint_interval=interval, ttl=5.0) for _ in range(n)]


def test_train_through_pservers_and_resume(store, tmp_path):
    servers = _servers(store, tmp_path)
    try:
        c0, c1 = ps.PServerClient(store, 2, trainer_id=0), ps.PServerClient(store, 2, trainer_id=1)
        assert c0.begin_init_params() and not c1.begin_init_params()
        rng = np.random.RandomState(0)
        params = {"w_sgd": rng.randn(4, 3).astype("float32"), "w_mom": rng.randn(5).astype("float32"),
                  "w_adam": rng.randn(3, 3).astype("float32"), "w_ada": rng.randn(6).astype("float32")}
        cfgs = {"w_sgd": {"optimizer": "sgd", "lr": 0.1},
                "w_mom": {"optimizer": "sgd", "lr": 0.1, "momentum": 0.9, "nesterov": True},
                "w_adam": {"optimizer": "adam", "lr": 0.01},
                "w_ada": {"optimizer": "adagrad", "lr": 0.5, "lr_policy": "linear", "lr_decay_a": 0.01,
                          "lr_decay_b": 0.1}}
        for n, v in params.items():
            c0.init_param(n, v, cfgs[n])
        c0.finish_init_params()
        assert {c0.partition(n) for n in params} == {0, 1}  # spread over both servers
        grads = [{n: rng.randn(*v.shape).astype("float32") for n, v in params.items()} for _ in range(3)]
        for g in grads:
            c1.send_grads(g, num_samples=8)
        got = c1.get_params(list(params))
        # reference updates
        w = params["w_sgd"].copy()
        for g in grads:
            w -= 0.1 * g["w_sgd"]
        np.testing.assert_allclose(got["w_sgd"], w, rtol=1e-6)
        w, vel = params["w_mom"].copy(), np.zeros(5, "float32")
        for g in grads:
            vel = 0.9 * vel - 0.1 * g["w_mom"]
            w += 0.9 * vel - 0.1 * g["w_mom"]
        np.testing.assert_allclose(got["w_mom"], w, rtol=1e-5)
        w, m, v = params["w_adam"].copy(), np.zeros((3, 3)), np.zeros((3, 3))
        for t, g in enumerate(grads, 1):
            m = 0.9 * m + 0.1 * g["w_adam"]
            v = 0.999 * v + 0.001 * g["w_adam"] ** 2
            w -= 0.01 * np.sqrt(1 - 0.999 ** t) / (1 - 0.9 ** t) * m / (np.sqrt(v) + 1e-8)
        np.testing.assert_allclose(got["w_adam"], w, rtol=1e-5)
        w, acc, samples = params["w_ada"].copy(), np.zeros(6), 0
        for g in grads:
            samples += 8
            lr = max(0.5 - 0.01 * samples, 0.1)
            acc += g["w_ada"] ** 2
            w -= lr * g["w_ada"] / (np.sqrt(acc) + 1e-6)
        np.testing.assert_allclose(got["w_ada"], w, rtol=1e-5)

        # checkpoint every server, kill server 0, start a replacement: it takes the
        # free slot 0, resumes from the CRC-checked checkpoint, optimizer state included
        for s in servers:
            s.service.checkpoint()
        dead = servers[0]
        dead.stop()
        servers[0] = ps.PServer(store, 2, str(tmp_path / "ckpt"), checkpoint_interval=0.0, ttl=5.0)
        assert servers[0].service.index == 0
        c1.reconnect()
        after = c1.get_params(list(params))
        for n in params:
            np.testing.assert_array_equal(after[n], got[n])
        g4 = {n: rng.randn(*v.shape).astype("float32") for n, v in params.items()}
        c1.send_grads(g4, num_samples=8)
        m = 0.9 * m + 0.1 * g4["w_adam"]
        v = 0.999 * v + 0.001 * g4["w_adam"] ** 2
        w_adam = got["w_adam"] - 0.01 * np.sqrt(1 - 0.999 ** 4) / (1 - 0.9 ** 4) * m / (np.sqrt(v) + 1e-8)
        np.testing.assert_allclose(c1.get_params(["w_adam"])["w_adam"], w_adam, rtol=1e-5)
        c0.close()
        c1.close()
    finally:
        for s in servers:
            s.stop()


def test_periodic_checkpoint_and_crc(store, tmp_path):
    servers = _servers(store, tmp_path, n=1, interval=0.2)
    try:
        c = ps.PServerClient(store, 1)
        c.init_param("w", np.ones(4, "float32"), {"optimizer": "sgd", "lr": 1.0})
        c.finish_init_params()
        c.send_grads({"w": np.full(4, 0.5, "float32")})
        t0 = time.time()
        while servers[0].service.last_checkpoint is None and time.time() - t0 < 5:
            time.sleep(0.05)
        info = store.get("/checkpoint/0")
        assert info and os.path.exists(info["path"])
        cp = ps.load_checkpoint(store, 0)
        np.testing.assert_array_equal(cp["w"][0], np.full(4, 0.5, "float32"))
        servers[0].service.shutdown()  # stop the periodic writer before corrupting
        time.sleep(0.3)
        info = store.get("/checkpoint/0")
        raw = bytearray(open(info["path"], "rb").read())
        raw[len(raw) // 2] ^= 0xFF
        open(info["path"], "wb").write(bytes(raw))
        with pytest.raises(ValueError, match="checksum"):
            ps.load_checkpoint(store, 0)
        c.close()
    finally:
        for s in servers:
            s.stop()
