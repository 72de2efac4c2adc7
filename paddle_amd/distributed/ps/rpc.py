"""ctypes bindings of the native PS transport (csrc/runtime/rpc.cc) plus the
variable (de)serialisation used on the wire (framework LoDTensor / SelectedRows
streams -- the same bytes the reference's sendrecvop_utils produces for
checkpoints)."""
from __future__ import annotations

import ctypes
import io
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

from ... import runtime
from ...framework import core
from ...framework import serialization as S

_P, _I, _SZ, _C = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_char_p
_PP = ctypes.POINTER(ctypes.c_void_p)
_SIGS = {
    "pa_rpc_server_create": ([ctypes.c_char_p, _I, _I], _P),
    "pa_rpc_server_port": ([_P], _I),
    "pa_rpc_server_wait": ([_P, _I, _I], _I),
    "pa_rpc_server_pop": ([_P, _PP, _PP, ctypes.POINTER(_SZ)], _I),
    "pa_rpc_server_pop_checkpoint": ([_P, _PP], _I),
    "pa_rpc_server_publish": ([_P, _C, _P, _SZ], _I),
    "pa_rpc_server_set_table": ([_P, _C, _P, _P, ctypes.c_int64, ctypes.c_int64], _I),
    "pa_rpc_server_set_ready": ([_P, _I], _I),
    "pa_rpc_server_reset_barriers": ([_P, _I], _I),
    "pa_rpc_server_stop": ([_P], _I),
    "pa_rpc_send": ([_C, _C, _P, _SZ], _I),
    "pa_rpc_get": ([_C, _C, _PP, ctypes.POINTER(_SZ)], _I),
    "pa_rpc_prefetch": ([_C, _C, _P, _SZ, _PP, ctypes.POINTER(_SZ)], _I),
    "pa_rpc_barrier": ([_C, _I], _I),
    "pa_rpc_checkpoint_notify": ([_C, _C], _I),
    "pa_rpc_free": ([_P], None),
    "pa_rpc_close_all": ([], _I),
}
_lib = None
_lock = threading.Lock()


def lib():
    global _lib
    with _lock:
        if _lib is None:
            L = runtime.lib()
            for n, (a, r) in _SIGS.items():
                f = getattr(L, n)
                f.argtypes, f.restype = a, r
            _lib = L
    return _lib


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: {runtime.lib().pa_rt_last_error().decode()}")


def _take(ptr, n):
    b = ctypes.string_at(ptr, n) if n else b""
    lib().pa_rpc_free(ptr)
    return b


# ------------------------------------------------------------------ serialisation
def var_to_bytes(v):
    if isinstance(v, core.SelectedRows):
        f = io.BytesIO()
        S.write_selected_rows(f, v)
        return b"S" + f.getvalue()
    if torch.is_tensor(v):
        v = core.LoDTensor(v)
    return b"T" + S.lod_tensor_to_bytes(v)


def bytes_to_var(b):
    if b[:1] == b"S":
        return S.read_selected_rows(io.BytesIO(b[1:]))
    return S.lod_tensor_from_bytes(b[1:])


# ------------------------------------------------------------------------ client
class RPCClient:
    """Process-wide client; calls fan out over a thread pool (the ctypes calls run
    with the GIL released), mirroring the reference's async Send/Get + Wait."""

    _inst = None

    @classmethod
    def instance(cls):
        if cls._inst is None:
            cls._inst = RPCClient()
        return cls._inst

    def __init__(self):
        self.pool = ThreadPoolExecutor(max_workers=16)
        self.futs = []
        self.endpoints = set()  # pservers this trainer sent to (notified on Executor.close)

    def _send(self, ep, name, data):
        buf = ctypes.create_string_buffer(data, len(data))
        _check(lib().pa_rpc_send(ep.encode(), name.encode(), buf, len(data)), f"send {name} -> {ep}")

    def _get(self, ep, name):
        out, n = ctypes.c_void_p(), _SZ()
        _check(lib().pa_rpc_get(ep.encode(), name.encode(), ctypes.byref(out), ctypes.byref(n)), f"get {name} <- {ep}")
        return _take(out, n.value)

    def async_send_var(self, ep, name, value):
        self.endpoints.add(ep)
        self.futs.append(self.pool.submit(self._send, ep, name, var_to_bytes(value)))

    def async_get_var(self, ep, name, callback):
        self.futs.append(self.pool.submit(lambda: callback(bytes_to_var(self._get(ep, name)))))

    def prefetch(self, ep, table, ids):
        ids = np.ascontiguousarray(np.asarray(ids, dtype=np.int64).reshape(-1))
        out, n = ctypes.c_void_p(), _SZ()
        _check(lib().pa_rpc_prefetch(ep.encode(), table.encode(), ids.ctypes.data, ids.size, ctypes.byref(out),
                                     ctypes.byref(n)), f"prefetch {table} <- {ep}")
        return np.frombuffer(_take(out, n.value), dtype=np.float32)

    def barrier(self, eps, kind):
        fs = [self.pool.submit(lambda e=e: _check(lib().pa_rpc_barrier(e.encode(), kind), f"barrier -> {e}"))
              for e in eps]
        for f in fs:
            f.result()

    def checkpoint_notify(self, eps, dirname):
        for e in eps:
            _check(lib().pa_rpc_checkpoint_notify(e.encode(), dirname.encode()), f"checkpoint -> {e}")

    def wait(self):
        fs, self.futs = self.futs, []
        for f in fs:
            f.result()

    def complete(self, eps):
        self.wait()
        self.barrier(eps, 2)


# ------------------------------------------------------------------------ server
class RPCServer:
    def __init__(self, port, fanin, host=None):
        """``host``: bind address (the pserver endpoint's host); None = all interfaces."""
        self.h = lib().pa_rpc_server_create((host or "").encode(), int(port), int(fanin))
        if not self.h:
            raise RuntimeError(runtime.lib().pa_rt_last_error().decode())
        self.port = lib().pa_rpc_server_port(self.h)

    def wait(self, what, timeout_ms=-1):
        return lib().pa_rpc_server_wait(self.h, what, timeout_ms)

    def pop_all(self):
        out = []
        while True:
            nm, data, n = ctypes.c_void_p(), ctypes.c_void_p(), _SZ()
            if not lib().pa_rpc_server_pop(self.h, ctypes.byref(nm), ctypes.byref(data), ctypes.byref(n)):
                return out
            name = ctypes.string_at(nm).decode()
            lib().pa_rpc_free(nm)
            out.append((name, bytes_to_var(_take(data, n.value))))

    def pop_checkpoints(self):
        out = []
        while True:
            d = ctypes.c_void_p()
            if not lib().pa_rpc_server_pop_checkpoint(self.h, ctypes.byref(d)):
                return out
            out.append(ctypes.string_at(d).decode())
            lib().pa_rpc_free(d)

    def publish(self, name, value):
        b = var_to_bytes(value)
        buf = ctypes.create_string_buffer(b, len(b))
        _check(lib().pa_rpc_server_publish(self.h, name.encode(), buf, len(b)), f"publish {name}")

    def set_table(self, name, ids, rows):
        ids = np.ascontiguousarray(np.asarray(ids, np.int64))
        rows = np.ascontiguousarray(np.asarray(rows, np.float32))
        _check(lib().pa_rpc_server_set_table(self.h, name.encode(), ids.ctypes.data, rows.ctypes.data, len(ids),
                                             rows.shape[1] if rows.ndim == 2 else 1), f"set_table {name}")

    def set_ready(self, ready):
        lib().pa_rpc_server_set_ready(self.h, 1 if ready else 0)

    def reset(self, which=3):
        lib().pa_rpc_server_reset_barriers(self.h, which)

    def stop(self):
        if self.h:
            lib().pa_rpc_server_stop(self.h)
            self.h = None
