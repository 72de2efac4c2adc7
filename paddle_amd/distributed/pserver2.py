"""Block-sharded parameter server of the legacy engine (reference
paddle/legacy/pserver/ParameterServer2.{h,cpp}, ParameterClient2.cpp,
proto/ParameterService.proto) -- the "old" pserver that v2 ``trainer.SGD(is_local=
False, use_etcd=False, pserver_spec=...)`` and the v1 trainer's remote updater talk
to (the Go-service counterpart is ``distributed/pserver.py``).

Layout (as ParameterClient2): every parameter is cut into blocks of
``parameter_block_size`` elements (``calc_block_size``: the per-server share rounded
to a power of two, >= 2^10, at most ~2^7 blocks per server; sparse-remote-update
parameters use one row per block); block ``b`` of parameter ``name`` lives on server
``(b + fnv1a32(name)) % num_servers``.

Update modes of ``send_parameter`` (ParameterService.proto ParameterUpdateMode):
* ``SET_PARAM`` / ``SET_PARAM_ZERO``: the initial values (trainer 0), then
  ``set_status(PARAMETER_READY)``;
* ``ADD_GRADIENT`` (synchronous SGD): every trainer adds its gradient blocks; the
  request carrying ``BATCH_FINISH`` blocks until all ``num_trainers`` trainers have
  finished the batch, the server then applies its optimizer (OptimizationConfig:
  sgd / momentum / adam / adagrad / adadelta) once to the averaged gradient and every
  waiting trainer gets the new values back (the gradientReady / parameterReady
  barrier pair of ParameterServer2::addGradient);
* ``ASYNC_SGD``: the gradient is applied at once; a trainer more than
  ``async_lagged_grad_discard_ratio * num_trainers`` updates behind is discarded
  (asyncGrdientCommitCheckAndStat);
* ``AVERAGE_PARAMETER``: the trainers' values are averaged (model averaging);
* ``GET_PARAM`` / ``GET_PARAM_SPARSE``: values (of the listed rows).
``synchronize`` is the trainers' barrier; ``save_value`` / ``load_value`` write each
server's blocks to ``save_dir`` (the per-server value vectors of saveValueVector).

Transport: a TCP connection per (client, server); a frame is the function name,
the request message in protobuf wire format (schemas below, encoded by
``trainer_config_helpers.config_proto``) and the data blocks as raw float32 iovecs --
the shape of the reference's ProtoServer / SocketChannel messages.
"""
from __future__ import annotations

import os
import socket
import socketserver
import struct
import threading

import numpy as np

from ..trainer_config_helpers import config_proto as cp
from .pserver import _Optimizer, fnv1a32

SET_PARAM, SET_PARAM_ZERO, ASYNC_SGD, ADD_GRADIENT, AVERAGE_PARAMETER, GET_PARAM, GET_PARAM_SPARSE = range(7)
BATCH_START, BATCH_ON, BATCH_FINISH, BATCH_START_AND_FINISH = range(4)
PSERVER_STATUS_NOT_SET, PSERVER_STATUS_PARAMETER_READY = 0, 1

cp._S.update({
    "ParameterBlock": [("para_id", 1, "uint64", 0), ("block_id", 2, "uint64", 0), ("begin_pos", 3, "uint64", 0),
                       ("block_size", 4, "uint64", 0)],
    "SendParameterRequest": [
        ("update_mode", 1, "int32", 0), ("blocks", 2, "ParameterBlock", 1), ("send_back_parameter", 3, "bool", 0),
        ("num_samples", 4, "int64", 0), ("cost", 5, "double", 0), ("batch_status", 6, "int32", 0),
        ("trainer_id", 7, "int32", 0)],
    "SendParameterResponse": [("blocks", 1, "ParameterBlock", 1)],
    "SetConfigRequest": [
        ("param_configs", 1, "ParameterConfig", 1), ("opt_config", 2, "OptimizationConfig", 0),
        ("save_dir", 4, "string", 0), ("server_id", 5, "int32", 0), ("is_sparse_server", 6, "bool", 0)],
    "SynchronizeRequest": [("sync_object_id", 1, "int32", 0), ("trainer_id", 2, "int32", 0)],
    "SetStatusRequest": [("status", 1, "int32", 0)],
    "GetStatusResponse": [("status", 1, "int32", 0)],
    "SaveValueRequest": [("dir_name", 1, "string", 0)],
    "Empty": [],
})
for _m in ("ParameterBlock", "SendParameterRequest", "SendParameterResponse", "SetConfigRequest",
           "SynchronizeRequest", "SetStatusRequest", "GetStatusResponse", "SaveValueRequest", "Empty"):
    cp._FIELDS[_m] = {f[0]: f for f in cp._S[_m]}
    cp._BYNUM[_m] = {f[1]: f for f in cp._S[_m]}
cp._S["OptimizationConfig"] = cp._S["OptimizationConfig"] + [
    ("async_lagged_grad_discard_ratio", 37, "double", 0)]
cp._FIELDS["OptimizationConfig"] = {f[0]: f for f in cp._S["OptimizationConfig"]}
cp._BYNUM["OptimizationConfig"] = {f[1]: f for f in cp._S["OptimizationConfig"]}


# ---------------------------------------------------------------- framing
def _send_frame(sock, func, msg, payload, iovs=()):
    parts = [func.encode(), cp.encode(msg, payload)] + [np.ascontiguousarray(a, np.float32).tobytes() for a in iovs]
    head = struct.pack("<I", len(parts)) + b"".join(struct.pack("<Q", len(p)) for p in parts)
    sock.sendall(struct.pack("<Q", len(head)) + head + b"".join(parts))


def _recv_exact(sock, n):
    buf = bytearray(n)
    view, got = memoryview(buf), 0
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if not k:
            raise ConnectionError("pserver2: connection closed")
        got += k
    return bytes(buf)


def _recv_frame(sock):
    (hl,) = struct.unpack("<Q", _recv_exact(sock, 8))
    head = _recv_exact(sock, hl)
    (n,) = struct.unpack("<I", head[:4])
    lens = struct.unpack(f"<{n}Q", head[4:4 + 8 * n])
    parts = [_recv_exact(sock, ln) for ln in lens]
    return parts[0].decode(), parts[1], [np.frombuffer(p, np.float32) for p in parts[2:]]


def calc_block_size(sizes, num_servers):
    """ParameterClient2::calcParameterBlockSize."""
    per = max(int(sum(sizes)) // max(num_servers, 1), 1)
    return 1 << max(per.bit_length() - 7, 10)


def _opt_from_config(oc, pc):
    """Server-side optimizer settings of one parameter from OptimizationConfig."""
    method = oc.get("learning_method", "momentum")
    cfg = {"lr": float(oc.get("learning_rate", 0.01)) * float(pc.get("learning_rate", 1.0)),
           "decay": float(pc.get("decay_rate", 0.0) or oc.get("l2weight", 0.0) or 0.0)}
    if method in ("momentum", "sgd"):
        cfg.update(optimizer="sgd", momentum=float(pc.get("momentum", 0.0)))
    elif method == "adam":
        cfg.update(optimizer="adam", beta1=oc.get("adam_beta1", 0.9), beta2=oc.get("adam_beta2", 0.999),
                   epsilon=oc.get("adam_epsilon", 1e-8))
    elif method == "adagrad":
        cfg.update(optimizer="adagrad", epsilon=oc.get("ada_epsilon", 1e-6))
    elif method == "adadelta":
        cfg.update(optimizer="adadelta", rho=oc.get("ada_rou", 0.95), epsilon=oc.get("ada_epsilon", 1e-6))
    else:
        raise ValueError(f"pserver2: unsupported learning_method {method}")
    return cfg


# ---------------------------------------------------------------- server
class _Block:
    __slots__ = ("value", "grad", "opt", "avg")

    def __init__(self, n):
        self.value = np.zeros(n, np.float32)
        self.grad = np.zeros(n, np.float32)
        self.opt = None
        self.avg = None


class ParameterServer2:
    """One server process / thread (``start()`` listens; ``port`` after start)."""

    def __init__(self, host="127.0.0.1", port=0, num_trainers=1):
        self.host, self.port, self.num_trainers = host, port, int(num_trainers)
        self.configs = {}      # para_id -> ParameterConfig dict
        self.opt_config = {}
        self.server_id = 0
        self.save_dir = ""
        self.blocks = {}       # (para_id, block_id) -> _Block
        self.status = PSERVER_STATUS_NOT_SET
        self._lock = threading.Lock()
        self._cv = threading.Condition(self._lock)
        self._finished = 0     # trainers that finished the current batch
        self._round = 0        # completed synchronous updates
        self._avg_count = 0
        self._avg_round = 0
        self._sync_count = 0
        self._sync_round = 0
        self.async_steps = 0
        self.trainer_steps = {}
        self.lagged_discarded = 0
        self.samples = 0
        self.cost = 0.0
        self._srv = None

    # -- lifecycle
    def start(self):
        srv = self

        class _H(socketserver.BaseRequestHandler):
            def handle(self):
                self.request.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                try:
                    while True:
                        func, msg, data = _recv_frame(self.request)
                        rmsg, rpay, riovs = srv.dispatch(func, msg, data)
                        _send_frame(self.request, func, rmsg, rpay, riovs)
                except (ConnectionError, OSError):
                    return

        class _S(socketserver.ThreadingMixIn, socketserver.TCPServer):
            daemon_threads = True
            allow_reuse_address = True

        self._srv = _S((self.host, self.port), _H)
        self.port = self._srv.server_address[1]
        threading.Thread(target=self._srv.serve_forever, daemon=True).start()
        return self

    def stop(self):
        if self._srv is not None:
            self._srv.shutdown()
            self._srv.server_close()
            self._srv = None

    # -- RPC dispatch
    def dispatch(self, func, msg, data):
        if func == "setConfig":
            r = cp.decode("SetConfigRequest", msg)
            with self._lock:
                self.configs = {i: c for i, c in enumerate(r.get("param_configs", []))}
                for c in r.get("param_configs", []):
                    if "para_id" in c:
                        self.configs[int(c["para_id"])] = c
                self.opt_config = r.get("opt_config", {})
                self.server_id = int(r.get("server_id", 0))
                self.save_dir = r.get("save_dir", "")
            return "Empty", {}, []
        if func == "sendParameter":
            return self.send_parameter(cp.decode("SendParameterRequest", msg), data)
        if func == "synchronize":
            self._barrier()
            return "Empty", {}, []
        if func == "setStatus":
            with self._cv:
                self.status = int(cp.decode("SetStatusRequest", msg).get("status", 0))
                self._cv.notify_all()
            return "Empty", {}, []
        if func == "getStatus":
            return "GetStatusResponse", {"status": self.status}, []
        if func == "waitPassStart" or func == "waitPassFinish":
            self._barrier()
            return "Empty", {}, []
        if func == "saveValueVector":
            self.save_value(cp.decode("SaveValueRequest", msg).get("dir_name") or self.save_dir)
            return "Empty", {}, []
        if func == "loadValueVector":
            self.load_value(cp.decode("SaveValueRequest", msg).get("dir_name") or self.save_dir)
            return "Empty", {}, []
        raise ValueError(f"pserver2: unknown function {func}")

    def _barrier(self):
        with self._cv:
            r = self._sync_round
            self._sync_count += 1
            if self._sync_count == self.num_trainers:
                self._sync_count = 0
                self._sync_round += 1
                self._cv.notify_all()
            else:
                while self._sync_round == r:
                    self._cv.wait()

    def _block(self, b, n, create=False):
        key = (int(b["para_id"]), int(b["block_id"]))
        blk = self.blocks.get(key)
        if blk is None:
            if not create:
                raise KeyError(f"pserver2: block {key} was never set")
            blk = self.blocks[key] = _Block(n)
        return key, blk

    def _optimizer(self, key, blk):
        if blk.opt is None:
            pc = self.configs.get(key[0], {})
            blk.opt = _Optimizer(blk.value, _opt_from_config(self.opt_config, pc))
        return blk.opt

    def send_parameter(self, req, data):
        mode = int(req.get("update_mode", 0))
        blocks = req.get("blocks", [])
        status = int(req.get("batch_status", BATCH_START_AND_FINISH))
        finish = status in (BATCH_FINISH, BATCH_START_AND_FINISH)
        out_blocks, out_data = [], []

        def reply():
            if req.get("send_back_parameter") or mode in (GET_PARAM, GET_PARAM_SPARSE):
                with self._lock:
                    for b in blocks:
                        _, blk = self._block(b, 0)
                        out_blocks.append(b)
                        out_data.append(blk.value.copy())
            return "SendParameterResponse", {"blocks": out_blocks}, out_data

        if mode in (SET_PARAM, SET_PARAM_ZERO):
            with self._lock:
                for i, b in enumerate(blocks):
                    n = int(b["block_size"])
                    _, blk = self._block(b, n, create=True)
                    blk.value[:] = 0.0 if mode == SET_PARAM_ZERO else data[i][:n]
                    blk.opt = None
            return reply()
        if mode in (GET_PARAM, GET_PARAM_SPARSE):
            return reply()
        if mode == ADD_GRADIENT:
            with self._cv:
                for i, b in enumerate(blocks):
                    _, blk = self._block(b, 0)
                    blk.grad += data[i][:blk.grad.size]
                if finish:
                    self.samples += int(req.get("num_samples", 0))
                    self.cost += float(req.get("cost", 0.0))
                    r = self._round
                    self._finished += 1
                    if self._finished == self.num_trainers:
                        # every trainer's gradient is in: one optimizer step on the average
                        inv = 1.0 / self.num_trainers
                        for key, blk in self.blocks.items():
                            g = blk.grad * inv
                            self._optimizer(key, blk).update(g, max(self.samples, 1))
                            blk.grad[:] = 0.0
                        self.samples, self._finished = 0, 0
                        self._round += 1
                        self._cv.notify_all()
                    else:
                        while self._round == r:
                            self._cv.wait()
            return reply()
        if mode == ASYNC_SGD:
            tid = int(req.get("trainer_id", 0))
            with self._lock:
                ratio = float(self.opt_config.get("async_lagged_grad_discard_ratio", 1.5))
                threshold = max(int(ratio * self.num_trainers), 1)
                lag = self.async_steps - self.trainer_steps.get(tid, 0)
                self.async_steps += 1
                if lag >= threshold:
                    self.lagged_discarded += 1
                else:
                    for i, b in enumerate(blocks):
                        key, blk = self._block(b, 0)
                        self._optimizer(key, blk).update(data[i][:blk.value.size], int(req.get("num_samples", 1)))
                self.trainer_steps[tid] = self.async_steps
            return reply()
        if mode == AVERAGE_PARAMETER:
            with self._cv:
                for i, b in enumerate(blocks):
                    _, blk = self._block(b, 0)
                    if blk.avg is None:
                        blk.avg = np.zeros_like(blk.value)
                    blk.avg += data[i][:blk.value.size]
                r = self._avg_round
                self._avg_count += 1
                if self._avg_count == self.num_trainers:
                    for blk in self.blocks.values():
                        if blk.avg is not None:
                            blk.value[:] = blk.avg / self.num_trainers
                            blk.avg = None
                    self._avg_count = 0
                    self._avg_round += 1
                    self._cv.notify_all()
                else:
                    while self._avg_round == r:
                        self._cv.wait()
            return reply()
        raise ValueError(f"pserver2: unsupported update mode {mode}")

    # -- checkpoint (per-server value vectors)
    def save_value(self, d):
        os.makedirs(d, exist_ok=True)
        with self._lock:
            arrs = {f"{k[0]}_{k[1]}": b.value for k, b in self.blocks.items()}
        np.savez(os.path.join(d, f"pserver_{self.server_id}.npz"), **arrs)

    def load_value(self, d):
        with np.load(os.path.join(d, f"pserver_{self.server_id}.npz")) as z:
            with self._lock:
                for k in z.files:
                    pid, bid = map(int, k.split("_"))
                    v = z[k]
                    blk = self.blocks.setdefault((pid, bid), _Block(v.size))
                    blk.value[:] = v
                    blk.opt = None


# ---------------------------------------------------------------- client
class ParameterClient2:
    """The trainer side: block layout, one connection per server, parallel requests."""

    def __init__(self, pserver_spec, trainer_id=0, timeout=60.0):
        eps = pserver_spec.split(",") if isinstance(pserver_spec, str) else list(pserver_spec)
        self.servers = []
        for ep in eps:
            h, p = ep.rsplit(":", 1)
            s = socket.create_connection((h, int(p)), timeout=timeout)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            self.servers.append(s)
        self.trainer_id = int(trainer_id)
        self.timeout = float(timeout)
        self.names, self.sizes, self.shapes, self.sparse = [], {}, {}, {}
        self.block_size = {}

    def close(self):
        for s in self.servers:
            s.close()
        self.servers = []

    def _call_all(self, func, msgs, payloads, iovs):
        """Send one request per server (in parallel threads), gather the responses."""
        res = [None] * len(self.servers)
        errs = []

        def one(i):
            try:
                _send_frame(self.servers[i], func, msgs[i], payloads[i], iovs[i])
                res[i] = _recv_frame(self.servers[i])
            except Exception as e:  # surfaced below
                errs.append(e)

        ts = [threading.Thread(target=one, args=(i,)) for i in range(len(self.servers))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errs:
            raise errs[0]
        return res

    # -- layout
    def init(self, params, param_configs=None, opt_config=None, save_dir=""):
        """``params``: ordered {name: ndarray}; sets the servers' config (para_id =
        position) and, on trainer 0, the initial values; other trainers wait for
        PARAMETER_READY.  Returns the values every trainer starts from."""
        self.names = list(params)
        sizes = [int(np.asarray(v).size) for v in params.values()]
        dense = calc_block_size(sizes, len(self.servers))
        pcs = []
        for i, (n, v) in enumerate(params.items()):
            v = np.asarray(v)
            pc = dict((param_configs or {}).get(n, {}))
            self.sparse[n] = bool(pc.get("sparse_remote_update", False))
            bs = int(v.shape[-1]) if self.sparse[n] else dense
            pc.update(name=n, size=int(v.size), dims=[int(d) for d in v.shape], parameter_block_size=bs,
                      para_id=i)
            self.sizes[n], self.shapes[n], self.block_size[n] = int(v.size), v.shape, bs
            pcs.append(pc)
        oc = dict(opt_config or {"learning_method": "momentum", "learning_rate": 0.01})
        oc.setdefault("algorithm", "sgd")
        msgs = [{"param_configs": [{k: c[k] for k in c if k in cp._FIELDS["ParameterConfig"]} for c in pcs],
                 "opt_config": oc, "save_dir": save_dir, "server_id": i, "is_sparse_server": False}
                for i in range(len(self.servers))]
        self._call_all("setConfig", ["SetConfigRequest"] * len(self.servers), msgs, [[]] * len(self.servers))
        if self.trainer_id == 0:
            self.send_parameter(SET_PARAM, params)
            self._call_all("setStatus", ["SetStatusRequest"] * len(self.servers),
                           [{"status": PSERVER_STATUS_PARAMETER_READY}] * len(self.servers), [[]] * len(self.servers))
        else:
            import time

            deadline = time.monotonic() + self.timeout
            while True:
                st = self._call_all("getStatus", ["Empty"] * len(self.servers), [{}] * len(self.servers),
                                    [[]] * len(self.servers))
                if all(cp.decode("GetStatusResponse", r[1]).get("status") == PSERVER_STATUS_PARAMETER_READY
                       for r in st):
                    break
                if time.monotonic() > deadline:
                    raise TimeoutError(f"pserver2: trainer {self.trainer_id}: parameters not ready after "
                                       f"{self.timeout:.0f} s (trainer 0 sets them)")
                time.sleep(0.01)
        return self.get_parameters()

    def _server_of(self, name, block_id):
        return abs((block_id + fnv1a32(name)) % len(self.servers))

    def _plan(self, values=None, rows=None):
        """Per server: (blocks, iovs) covering every parameter (or the given rows of
        sparse parameters)."""
        S = len(self.servers)
        blocks = [[] for _ in range(S)]
        iovs = [[] for _ in range(S)]
        for pid, n in enumerate(self.names):
            size, bs = self.sizes[n], self.block_size[n]
            flat = None if values is None else np.ascontiguousarray(values[n], np.float32).reshape(-1)
            ids = rows.get(n) if rows is not None and n in rows else range((size + bs - 1) // bs)
            for b in ids:
                b = int(b)
                lo, hi = b * bs, min(b * bs + bs, size)
                s = self._server_of(n, b)
                blocks[s].append({"para_id": pid, "block_id": b, "begin_pos": lo, "block_size": hi - lo})
                if flat is not None:
                    iovs[s].append(flat[lo:hi])
        return blocks, iovs

    def send_parameter(self, mode, values=None, send_back=False, batch_status=BATCH_START_AND_FINISH,
                       num_samples=0, cost=0.0, rows=None):
        blocks, iovs = self._plan(values, rows)
        msgs = [{"update_mode": mode, "blocks": blocks[s], "send_back_parameter": bool(send_back),
                 "num_samples": int(num_samples), "cost": float(cost), "batch_status": batch_status,
                 "trainer_id": self.trainer_id} for s in range(len(self.servers))]
        res = self._call_all("sendParameter", ["SendParameterRequest"] * len(self.servers), msgs, iovs)
        if not (send_back or mode in (GET_PARAM, GET_PARAM_SPARSE)):
            return None
        out = {n: np.zeros(self.sizes[n], np.float32) for n in self.names} if rows is None else \
            {n: {} for n in rows}
        for func, msg, data in res:
            for b, d in zip(cp.decode("SendParameterResponse", msg).get("blocks", []), data):
                n = self.names[int(b["para_id"])]
                lo = int(b["begin_pos"])
                if rows is None:
                    out[n][lo:lo + int(b["block_size"])] = d
                else:
                    out[n][int(b["block_id"])] = d.copy()
        if rows is None:
            return {n: out[n].reshape(self.shapes[n]) for n in self.names}
        return out

    # -- trainer API
    def get_parameters(self):
        return self.send_parameter(GET_PARAM)

    def get_rows(self, rows):
        """{name: [row ids]} of sparse-remote-update parameters -> {name: {row: values}}."""
        return self.send_parameter(GET_PARAM_SPARSE, rows=rows)

    def add_gradient(self, grads, num_samples=0, cost=0.0):
        """Synchronous SGD step: returns the parameters after every trainer's gradient."""
        return self.send_parameter(ADD_GRADIENT, grads, send_back=True, batch_status=BATCH_START_AND_FINISH,
                                   num_samples=num_samples, cost=cost)

    def async_sgd(self, grads, num_samples=0):
        return self.send_parameter(ASYNC_SGD, grads, send_back=True, num_samples=num_samples)

    def average_parameters(self, values):
        return self.send_parameter(AVERAGE_PARAMETER, values, send_back=True)

    def synchronize(self):
        self._call_all("synchronize", ["SynchronizeRequest"] * len(self.servers),
                       [{"trainer_id": self.trainer_id}] * len(self.servers), [[]] * len(self.servers))

    def save_values(self, dir_name):
        self._call_all("saveValueVector", ["SaveValueRequest"] * len(self.servers),
                       [{"dir_name": dir_name}] * len(self.servers), [[]] * len(self.servers))

    def load_values(self, dir_name):
        self._call_all("loadValueVector", ["SaveValueRequest"] * len(self.servers),
                       [{"dir_name": dir_name}] * len(self.servers), [[]] * len(self.servers))


def main(argv=None):
    """``python -m paddle_amd.distributed.pserver2 --port P [--ports_num K]
    --num_gradient_servers N`` (ParameterServer2Main): K servers on ports P..P+K-1,
    serving N trainers, until interrupted."""
    import argparse
    import time

    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, default=20134)
    ap.add_argument("--ports_num", type=int, default=1)
    ap.add_argument("--num_gradient_servers", type=int, default=1, help="number of trainers")
    ap.add_argument("--host", default="127.0.0.1")
    a = ap.parse_args(argv)
    servers = [ParameterServer2(a.host, a.port + i, a.num_gradient_servers).start() for i in range(a.ports_num)]
    print("pserver2 listening on", ",".join(f"{a.host}:{s.port}" for s in servers), flush=True)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        for s in servers:
            s.stop()


if __name__ == "__main__":
    main()
