"""Elastic parameter server of the fault-tolerant v2 trainer (reference: go/pserver --
service.go, client/client.go, etcd_client.go, optimizer.go -> the C++
paddle/optimizer library).

* ``PServerService``: ``init_param`` (parameter + optimizer config) ...
  ``finish_init_params`` (then a checkpoint thread runs every ``checkpoint_interval``),
  ``send_grad`` applies the parameter's optimizer, ``get_param``.  Checkpoints hold
  every parameter, its config and its optimizer state; the file is written
  atomically, its CRC32 + path + timestamp go to the KV store under
  ``/checkpoint/<index>``, and a restarted server resumes from it
  (``load_checkpoint`` verifies the CRC).
* optimizers (the "cgo optimizer" row): SGD (momentum / Nesterov / decay), Adam,
  Adagrad, Adadelta; learning-rate policies "const" and "linear"
  (lr = max(lr - a * samples, b)).  State serialises to plain arrays (no pickle).
* registration / discovery (the etcd row): ``KVStore`` is a lock-protected JSON
  file with leases (``ttl``): ``register_pserver`` claims the lowest free
  ``/ps/<i>`` slot below ``/ps_desired`` and a keep-alive thread refreshes it;
  ``list_pservers`` returns the live slots; a dead server's slot expires and the
  replacement takes the same index (and its checkpoint).
* ``PServerClient``: partitions parameters over servers by FNV-1a(name) % n (as the
  Go client), ``begin_init_params`` elects the one trainer that initialises,
  ``send_grads`` fans out in parallel, reconnects when the listed address changes.

Transport: line-delimited JSON over TCP (as distributed/master.py), tensors base64.
"""
from __future__ import annotations

import base64
import fcntl
import io
import json
import os
import threading
import time
import uuid
import zlib

import numpy as np

from .master import MasterClient, MasterServer  # noqa: F401  (same TCP transport)

# ------------------------------------------------------------------ KV store with leases (etcd)


class KVStore:
    def __init__(self, path):
        self.path = path
        os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)

    def _txn(self, fn):
        with open(self.path + ".lock", "a+") as lk:
            fcntl.flock(lk, fcntl.LOCK_EX)
            try:
                d = {}
                if os.path.exists(self.path):
                    with open(self.path) as f:
                        d = json.load(f)
                now = time.time()
                d = {k: v for k, v in d.items() if v.get("exp") is None or v["exp"] > now}
                out, changed = fn(d)
                if changed:
                    tmp = self.path + ".tmp"
                    with open(tmp, "w") as f:
                        json.dump(d, f)
                    os.replace(tmp, self.path)
                return out
            finally:
                fcntl.flock(lk, fcntl.LOCK_UN)

    def get(self, key):
        return self._txn(lambda d: (d[key]["v"] if key in d else None, False))

    def put(self, key, value, ttl=None):
        def fn(d):
            d[key] = {"v": value, "exp": (time.time() + ttl) if ttl else None}
            return True, True
        return self._txn(fn)

    def put_if_absent(self, key, value, ttl=None):
        def fn(d):
            if key in d:
                return False, False
            d[key] = {"v": value, "exp": (time.time() + ttl) if ttl else None}
            return True, True
        return self._txn(fn)

    def refresh(self, key, ttl):
        def fn(d):
            if key not in d:
                return False, False
            d[key]["exp"] = time.time() + ttl
            return True, True
        return self._txn(fn)

    def delete(self, key):
        return self._txn(lambda d: (d.pop(key, None) is not None, True))

    def list(self, prefix):
        return self._txn(lambda d: ({k: v["v"] for k, v in d.items() if k.startswith(prefix)}, False))


class Registration:
    """A claimed ``/ps/<index>`` slot kept alive by a refresh thread (etcd session)."""

    def __init__(self, store, index, ttl):
        self.store, self.index, self.ttl = store, index, ttl
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._keepalive, daemon=True)
        self._t.start()

    def _keepalive(self):
        while not self._stop.wait(self.ttl / 3):
            self.store.refresh(f"/ps/{self.index}", self.ttl)

    def close(self, release=True):
        self._stop.set()
        if release:
            self.store.delete(f"/ps/{self.index}")


def register_pserver(store, num_pservers, endpoint, ttl=10.0, timeout=30.0):
    """Claim the lowest free pserver index (etcd_client.go Register)."""
    store.put_if_absent("/ps_desired", int(num_pservers))
    desired = int(store.get("/ps_desired"))
    t0 = time.time()
    while True:
        for i in range(desired):
            if store.put_if_absent(f"/ps/{i}", endpoint, ttl=ttl):
                return Registration(store, i, ttl)
        if time.time() - t0 > timeout:
            raise TimeoutError(f"no free pserver slot among {desired}")
        time.sleep(0.1)


def list_pservers(store):
    """[(index, address)] of the live pservers (the client's Lister)."""
    out = []
    for k, v in store.list("/ps/").items():
        out.append((int(k.rsplit("/", 1)[1]), v))
    return sorted(out)


# ------------------------------------------------------------------ optimizers ("cgo optimizer")


class _Optimizer:
    def __init__(self, param, config, state=None):
        self.p = param
        self.cfg = dict(config)
        self.kind = self.cfg.get("optimizer", "sgd")
        self.t = 0
        self.samples = 0
        self.st = {}
        if self.kind == "sgd" and self.cfg.get("momentum", 0.0):
            self.st["vel"] = np.zeros_like(param)
        elif self.kind == "adam":
            self.st["m"], self.st["v"] = np.zeros_like(param), np.zeros_like(param)
        elif self.kind == "adagrad":
            self.st["acc"] = np.zeros_like(param)
        elif self.kind == "adadelta":
            self.st["eg"], self.st["ex"] = np.zeros_like(param), np.zeros_like(param)
        elif self.kind != "sgd":
            raise ValueError(f"unknown optimizer {self.kind}")
        if state:
            self.t, self.samples = int(state["t"]), int(state["samples"])
            for k in self.st:
                self.st[k] = state[k].astype(param.dtype).reshape(param.shape)

    def lr(self):
        c = self.cfg
        base = float(c.get("lr", 0.01))
        if c.get("lr_policy", "const") == "linear":
            return max(base - float(c.get("lr_decay_a", 0.0)) * self.samples, float(c.get("lr_decay_b", 0.0)))
        return base

    def update(self, g, num_samples=1):
        c, p = self.cfg, self.p
        self.t += 1
        self.samples += int(num_samples)
        lr = self.lr()
        decay = float(c.get("decay", 0.0))
        if decay:
            g = g + decay * p
        if self.kind == "sgd":
            mu = float(c.get("momentum", 0.0))
            if mu:
                v = self.st["vel"]
                v *= mu
                v -= lr * g
                p += (mu * v - lr * g) if c.get("nesterov", False) else v
            else:
                p -= lr * g
        elif self.kind == "adam":
            b1, b2, eps = float(c.get("beta1", 0.9)), float(c.get("beta2", 0.999)), float(c.get("epsilon", 1e-8))
            m, v = self.st["m"], self.st["v"]
            m *= b1
            m += (1 - b1) * g
            v *= b2
            v += (1 - b2) * g * g
            p -= lr * np.sqrt(1 - b2 ** self.t) / (1 - b1 ** self.t) * m / (np.sqrt(v) + eps)
        elif self.kind == "adagrad":
            a = self.st["acc"]
            a += g * g
            p -= lr * g / (np.sqrt(a) + float(c.get("epsilon", 1e-6)))
        else:  # adadelta
            rho, eps = float(c.get("rho", 0.95)), float(c.get("epsilon", 1e-6))
            eg, ex = self.st["eg"], self.st["ex"]
            eg *= rho
            eg += (1 - rho) * g * g
            dx = -np.sqrt((ex + eps) / (eg + eps)) * g
            ex *= rho
            ex += (1 - rho) * dx * dx
            p += lr * dx

    def state(self):
        out = {"t": np.array(self.t), "samples": np.array(self.samples)}
        out.update(self.st)
        return out


class _NativeOptimizer:
    """A parameter whose config carries ``optimizer_config`` (hex of a serialised
    OptimizerConfig): updated by the native optimizer library
    (csrc/runtime/param_optimizer.cc) -- the reference Go pserver's cgo optimizer."""

    def __init__(self, param, config, state=None):
        from .param_optimizer import ParameterOptimizer

        self.cfg = dict(config)
        self.p = np.ascontiguousarray(param, np.float32).copy()
        st = bytes(np.asarray(state["native"], np.uint8)) if state and "native" in state else None
        self._o = ParameterOptimizer(bytes.fromhex(self.cfg["optimizer_config"]), self.p, state=st)
        self.p[...] = self._o.weights()

    def update(self, g, num_samples=1):
        self._o.update(g)
        self.p[...] = self._o.weights()

    def state(self):
        return {"native": np.frombuffer(self._o.state(), np.uint8).copy()}


def _make_optimizer(param, config, state=None):
    if isinstance(config, dict) and "optimizer_config" in config:
        return _NativeOptimizer(param, config, state)
    return _Optimizer(param, config, state)


# ------------------------------------------------------------------ service


def _enc(a):
    return {"dtype": str(a.dtype), "shape": list(a.shape), "b64": base64.b64encode(a.tobytes()).decode()}


def _dec(d):
    return np.frombuffer(base64.b64decode(d["b64"]), dtype=np.dtype(d["dtype"])).reshape(d["shape"]).copy()


class PServerService:
    def __init__(self, index=0, checkpoint_interval=60.0, checkpoint_dir=None, store=None, checkpoint=None):
        self.index = index
        self.interval = float(checkpoint_interval)
        self.dir = checkpoint_dir
        self.store = store
        self._mu = threading.Lock()
        self._opt = {}
        self._initialized = threading.Event()
        self._stop = threading.Event()
        self._ckpt_thread = None
        self.last_checkpoint = None
        if checkpoint is not None:  # resume (service.go NewService with a checkpoint)
            for name, (param, cfg, state) in checkpoint.items():
                self._opt[name] = _make_optimizer(param, cfg, state)
            self._start()

    # -- RPCs
    def init_param(self, name, param, config):
        if self._initialized.is_set():
            raise RuntimeError("parameters already initialized")
        with self._mu:
            self._opt[name] = _make_optimizer(_dec(param), config)
        return True

    def finish_init_params(self):
        if self._initialized.is_set():
            raise RuntimeError("parameters already initialized")
        self._start()
        return True

    def send_grad(self, name, grad, num_samples=1):
        if not self._initialized.is_set():
            raise RuntimeError("received gradient before initialization")
        with self._mu:
            o = self._opt.get(name)
            if o is None:
                raise KeyError(f"parameter {name} does not exist")
            o.update(_dec(grad).astype(o.p.dtype).reshape(o.p.shape), num_samples)
        return True

    def get_param(self, name):
        self._initialized.wait()
        with self._mu:
            o = self._opt.get(name)
            if o is None:
                raise KeyError(f"parameter {name} does not exist")
            return _enc(o.p)

    def status(self):
        return {"index": self.index, "initialized": self._initialized.is_set(), "params": sorted(self._opt)}

    # -- checkpointing
    def _start(self):
        self._initialized.set()
        if self.dir and self.interval > 0 and self._ckpt_thread is None:
            self._ckpt_thread = threading.Thread(target=self._ckpt_loop, daemon=True)
            self._ckpt_thread.start()

    def _ckpt_loop(self):
        while not self._stop.wait(self.interval):
            try:
                self.checkpoint()
            except Exception:  # noqa: BLE001  (logged by the next successful one)
                pass

    def checkpoint(self):
        with self._mu:
            arrays, meta = {}, {}
            for i, (name, o) in enumerate(sorted(self._opt.items())):
                arrays[f"p{i}"] = o.p.copy()
                for k, v in o.state().items():
                    arrays[f"s{i}_{k}"] = np.asarray(v)
                meta[name] = {"i": i, "config": o.cfg, "state_keys": list(o.state())}
        buf = io.BytesIO()
        np.savez(buf, __meta__=np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8), **arrays)
        content = buf.getvalue()
        os.makedirs(self.dir, exist_ok=True)
        path = os.path.join(self.dir, f"pserver_{self.index}_{uuid.uuid4().hex}.ckpt")
        with open(path + ".tmp", "wb") as f:
            f.write(content)
            f.flush()
            os.fsync(f.fileno())
        os.replace(path + ".tmp", path)
        info = {"uuid": os.path.basename(path), "path": path, "crc32": zlib.crc32(content) & 0xFFFFFFFF,
                "timestamp": time.time()}
        old = self.store.get(f"/checkpoint/{self.index}") if self.store else None
        if self.store:
            self.store.put(f"/checkpoint/{self.index}", info)
        if old and old.get("path") != path and os.path.exists(old["path"]):
            os.remove(old["path"])
        self.last_checkpoint = info
        return info

    def shutdown(self):
        self._stop.set()


def load_checkpoint(store, index):
    """{name: (param, config, state)} of pserver ``index`` or None (service.go
    LoadCheckpoint); raises on a CRC mismatch."""
    info = store.get(f"/checkpoint/{index}")
    if not info:
        return None
    with open(info["path"], "rb") as f:
        content = f.read()
    if zlib.crc32(content) & 0xFFFFFFFF != info["crc32"]:
        raise ValueError(f"checkpoint {info['path']}: checksum validation failed")
    z = np.load(io.BytesIO(content), allow_pickle=False)
    meta = json.loads(bytes(z["__meta__"]).decode())
    out = {}
    for name, m in meta.items():
        i = m["i"]
        out[name] = (z[f"p{i}"].copy(), m["config"], {k: z[f"s{i}_{k}"] for k in m["state_keys"]})
    return out


class PServer:
    """A service on TCP, registered in the store (cmd/pserver main of the reference)."""

    def __init__(self, store, num_pservers, checkpoint_dir, checkpoint_interval=60.0, ttl=10.0, host="127.0.0.1"):
        # serve first to know the port, then claim a slot and (maybe) resume
        self.service = PServerService(checkpoint_interval=checkpoint_interval, checkpoint_dir=checkpoint_dir,
                                      store=store)
        self.server = MasterServer(self.service, host=host)
        self.reg = register_pserver(store, num_pservers, self.server.endpoint, ttl=ttl)
        self.service.index = self.reg.index
        cp = load_checkpoint(store, self.reg.index)
        if cp is not None:
            for name, (param, cfg, state) in cp.items():
                self.service._opt[name] = _make_optimizer(param, cfg, state)
            self.service._start()
        self.endpoint = self.server.endpoint

    def stop(self, release=True):
        self.reg.close(release)
        self.server.stop()


# ------------------------------------------------------------------ client


def fnv1a32(s: str) -> int:
    h = 0x811C9DC5
    for b in s.encode():
        h ^= b
        h = (h * 0x01000193) & 0xFFFFFFFF
    return h


class _PSConn(MasterClient):
    _RPC = ("init_param", "finish_init_params", "send_grad", "get_param", "status")


class PServerClient:
    def __init__(self, store, num_pservers, trainer_id=0, timeout=30.0):
        self.store, self.n, self.trainer_id = store, int(num_pservers), trainer_id
        self._conns = [None] * self.n
        self._addrs = [None] * self.n
        self._wait(timeout)

    def _wait(self, timeout):
        t0 = time.time()
        while True:
            live = dict(list_pservers(self.store))
            if all(i in live for i in range(self.n)):
                break
            if time.time() - t0 > timeout:
                raise TimeoutError(f"pservers {sorted(set(range(self.n)) - set(live))} not registered")
            time.sleep(0.05)
        self._refresh(live)

    def _refresh(self, live=None):
        live = live if live is not None else dict(list_pservers(self.store))
        for i in range(self.n):
            addr = live.get(i)
            if addr and addr != self._addrs[i]:
                if self._conns[i] is not None:
                    self._conns[i].close()
                self._conns[i] = _PSConn(addr)
                self._addrs[i] = addr

    def partition(self, name):
        return fnv1a32(name) % self.n

    def _conn(self, name):
        return self._conns[self.partition(name)]

    def begin_init_params(self):
        """True for the one trainer that initialises the parameters (Selector)."""
        return bool(self.store.put_if_absent("/init_params_owner", self.trainer_id))

    def init_param(self, name, value, config):
        return self._conn(name).init_param(name, _enc(np.ascontiguousarray(value)), config)

    def finish_init_params(self):
        for c in self._conns:
            c.finish_init_params()
        return True

    def send_grads(self, grads, num_samples=1):
        errs = []

        def one(name, g):
            try:
                self._conn(name).send_grad(name, _enc(np.ascontiguousarray(g)), num_samples)
            except Exception as e:  # noqa: BLE001
                errs.append(e)

        ts = [threading.Thread(target=one, args=(n, g)) for n, g in grads.items()]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errs:
            raise errs[0]

    def get_params(self, names):
        return {n: _dec(self._conn(n).get_param(n)) for n in names}

    def reconnect(self):
        self._refresh()

    def close(self):
        for c in self._conns:
            if c is not None:
                c.close()
