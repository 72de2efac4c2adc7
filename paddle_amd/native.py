"""ctypes bindings of the native C++ executor (csrc/native, libpaddle_amd_native.so).

The library is a standalone C++ framework core -- ProgramDesc decoding, scopes,
host kernels, gfx950 device kernels, the block executor and the
``paddle_inference_api.h`` predictor -- usable from C++ without Python
(csrc/native/demo_*.cc).  These bindings expose the same objects to Python so the
tests can compare the native path against the Python executor:

* ``NativePredictor(model_dir, ...)``: ``run([np arrays]) -> [np arrays]``
  (reference: inference/api/api_impl.cc NativePaddlePredictor);
* ``NativeProgram`` / ``NativeScope`` / ``NativeExecutor``: run any saved program
  (e.g. startup + training programs) in a native scope.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _build

_lib = None
_P, _I, _I64, _SZ = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_size_t
_DT_TO_NP = {5: np.float32, 3: np.int64, 2: np.int32, 6: np.float64, 0: np.bool_, 20: np.uint8}
_NP_TO_DT = {np.dtype(v): k for k, v in _DT_TO_NP.items()}
_PADDLE_DT = {np.dtype(np.float32): 0, np.dtype(np.int64): 1, np.dtype(np.int32): 2}  # PaddleDType
_PADDLE_DT_NP = {0: np.float32, 1: np.int64, 2: np.int32}


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_build.NATIVE_LIB):
            _build.build_native()
        L = ctypes.CDLL(_build.NATIVE_LIB)
        sig = {
            "pa_nat_last_error": ([], ctypes.c_char_p),
            "pa_nat_create": ([ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, _I, _I, _I], _P),
            "pa_nat_clone": ([_P], _P),
            "pa_nat_destroy": ([_P], None),
            "pa_nat_run": ([_P, _I, ctypes.POINTER(_I), ctypes.POINTER(_I), ctypes.POINTER(_I64),
                            ctypes.POINTER(_P), ctypes.POINTER(_I64), ctypes.POINTER(_I)], _I),
            "pa_nat_output": ([_P, _I, ctypes.POINTER(_I), ctypes.POINTER(_I), ctypes.POINTER(_I64), _I,
                               ctypes.POINTER(_P), ctypes.POINTER(_SZ)], _I),
            "pa_nat_program_load": ([ctypes.c_char_p], _P),
            "pa_nat_program_parse": ([ctypes.c_char_p, _SZ], _P),
            "pa_nat_program_free": ([_P], None),
            "pa_nat_program_num_ops": ([_P, _I], _I),
            "pa_nat_scope_new": ([], _P),
            "pa_nat_scope_free": ([_P], None),
            "pa_nat_executor_new": ([_I], _P),
            "pa_nat_executor_free": ([_P], None),
            "pa_nat_executor_run": ([_P, _P, _P, _I], _I),
            "pa_nat_scope_set": ([_P, ctypes.c_char_p, _I, _I, ctypes.POINTER(_I64), _P, _I], _I),
            "pa_nat_scope_get": ([_P, ctypes.c_char_p, ctypes.POINTER(_I), ctypes.POINTER(_I), ctypes.POINTER(_I64),
                                  _I, ctypes.POINTER(_P), ctypes.POINTER(_SZ)], _I),
            "pa_nat_scope_share": ([_P, ctypes.c_char_p, _I, _I, ctypes.POINTER(_I64), _P, _I], _I),
            "pa_nat_scope_info": ([_P, ctypes.c_char_p, ctypes.POINTER(_I), ctypes.POINTER(_I), ctypes.POINTER(_I64),
                                   _I, ctypes.POINTER(_P), ctypes.POINTER(_I)], _I),
            "pa_nat_copy": ([_P, _I, _P, _I, _SZ], _I),
            "pa_nat_executor_fallbacks": ([_P, ctypes.c_char_p, _I], _I),
            "pa_nat_load_persistables": ([_P, _P, ctypes.c_char_p, ctypes.c_char_p, _I], _I),
            "pa_nat_registered_ops": ([ctypes.c_char_p, _I, _I], _I),
            "pa_nat_device_sgemm": ([_P, _I, _I, _I64, _I64, _I64, ctypes.c_float, _P, _I64, _P, _I64,
                                     ctypes.c_float, _P, _I64], _I),
        }
        for n, (a, r) in sig.items():
            f = getattr(L, n)
            f.argtypes, f.restype = a, r
        _lib = L
    return _lib


def _err():
    m = lib().pa_nat_last_error()
    return m.decode() if m else "unknown error"


def _b(s):
    return s.encode() if s else None


def registered_ops(device=False):
    buf = ctypes.create_string_buffer(1 << 16)
    n = lib().pa_nat_registered_ops(buf, len(buf), 1 if device else 0)
    if n < 0:
        raise RuntimeError("op list does not fit")
    return buf.value.decode().split()


class NativePredictor:
    """C++ NativePaddlePredictor (``ir_optim``: the kAnalysis engine with fc fusion)."""

    def __init__(self, model_dir=None, prog_file=None, param_file=None, use_gpu=False, device=0, ir_optim=False,
                 _handle=None):
        self._h = _handle or lib().pa_nat_create(_b(model_dir), _b(prog_file), _b(param_file), int(bool(use_gpu)),
                                                 int(device), int(bool(ir_optim)))
        if not self._h:
            raise RuntimeError(f"native predictor: {_err()}")

    def clone(self):
        return NativePredictor(_handle=lib().pa_nat_clone(self._h))

    def run(self, inputs, lods=None):
        arrs = [np.ascontiguousarray(a) for a in inputs]
        n = len(arrs)
        dt = (_I * n)(*[_PADDLE_DT[a.dtype] for a in arrs])
        nd = (_I * n)(*[a.ndim for a in arrs])
        dims = [d for a in arrs for d in a.shape]
        dims_c = (_I64 * max(1, len(dims)))(*dims)
        data = (_P * n)(*[a.ctypes.data for a in arrs])
        lod_flat, lod_len = [], []
        for i in range(n):
            lv = (lods or [None] * n)[i]
            lod_len.append(len(lv) if lv else 0)
            lod_flat.extend(lv or [])
        lf = (_I64 * max(1, len(lod_flat)))(*lod_flat)
        ll = (_I * n)(*lod_len)
        k = lib().pa_nat_run(self._h, n, dt, nd, dims_c, data, lf, ll)
        if k < 0:
            raise RuntimeError(f"native predictor run: {_err()}")
        outs = []
        for i in range(k):
            t, nd1, p, nb = _I(), _I(), _P(), _SZ()
            d = (_I64 * 16)()
            if lib().pa_nat_output(self._h, i, ctypes.byref(t), ctypes.byref(nd1), d, 16, ctypes.byref(p),
                                   ctypes.byref(nb)) != 0:
                raise RuntimeError("native predictor: bad output index")
            shape = tuple(d[j] for j in range(nd1.value))
            buf = (ctypes.c_char * nb.value).from_address(p.value) if nb.value else b""
            outs.append(np.frombuffer(bytes(buf), dtype=_PADDLE_DT_NP[t.value]).reshape(shape).copy())
        return outs

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.pa_nat_destroy(self._h)
            self._h = None


class NativeProgram:
    def __init__(self, path=None, data: bytes | None = None):
        self._h = lib().pa_nat_program_load(path.encode()) if path else lib().pa_nat_program_parse(data, len(data))
        if not self._h:
            raise RuntimeError(f"native program: {_err()}")

    def num_ops(self, block=0):
        return lib().pa_nat_program_num_ops(self._h, block)

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.pa_nat_program_free(self._h)


class NativeScope:
    def __init__(self):
        self._h = lib().pa_nat_scope_new()

    def set(self, name, arr, device=-1):
        a = np.ascontiguousarray(arr)
        dims = (_I64 * max(1, a.ndim))(*a.shape)
        if lib().pa_nat_scope_set(self._h, name.encode(), _NP_TO_DT[a.dtype], a.ndim, dims, a.ctypes.data,
                                  int(device)) != 0:
            raise RuntimeError(_err())

    def get(self, name):
        t, nd, p, nb = _I(), _I(), _P(), _SZ()
        d = (_I64 * 16)()
        if lib().pa_nat_scope_get(self._h, name.encode(), ctypes.byref(t), ctypes.byref(nd), d, 16, ctypes.byref(p),
                                  ctypes.byref(nb)) != 0:
            raise RuntimeError(_err())
        shape = tuple(d[j] for j in range(nd.value))
        buf = (ctypes.c_char * nb.value).from_address(p.value) if nb.value else b""
        return np.frombuffer(bytes(buf), dtype=_DT_TO_NP[t.value]).reshape(shape).copy()

    def share(self, name, ptr, dtype_code, shape, device=-1):
        """Binds ``name`` to caller-owned memory (``ptr``, e.g. a torch tensor's
        storage): kernels update it in place, the executor never frees it."""
        dims = (_I64 * max(1, len(shape)))(*shape)
        if lib().pa_nat_scope_share(self._h, name.encode(), int(dtype_code), len(shape), dims, ptr, int(device)) != 0:
            raise RuntimeError(_err())

    def info(self, name):
        """(dtype code, shape, data pointer, device) of ``name``, or None."""
        t, nd, p, dev = _I(), _I(), _P(), _I()
        d = (_I64 * 16)()
        if not lib().pa_nat_scope_info(self._h, name.encode(), ctypes.byref(t), ctypes.byref(nd), d, 16,
                                       ctypes.byref(p), ctypes.byref(dev)):
            return None
        return t.value, tuple(d[j] for j in range(nd.value)), p.value or 0, dev.value

    def load_persistables(self, program: NativeProgram, dirname, combined=None, device=-1):
        if lib().pa_nat_load_persistables(program._h, self._h, _b(dirname), _b(combined), int(device)) != 0:
            raise RuntimeError(_err())

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.pa_nat_scope_free(self._h)


class NativeExecutor:
    def __init__(self, device=-1):
        self._h = lib().pa_nat_executor_new(int(device))
        if not self._h:
            raise RuntimeError(_err())

    def run(self, program: NativeProgram, scope: NativeScope, block=0):
        if lib().pa_nat_executor_run(self._h, program._h, scope._h, int(block)) != 0:
            raise RuntimeError(f"native executor: {_err()}")

    def host_fallbacks(self):
        """{op type: count} of ops this device executor ran on host copies."""
        buf = ctypes.create_string_buffer(1 << 16)
        n = lib().pa_nat_executor_fallbacks(self._h, buf, len(buf))
        if n < 0:
            raise RuntimeError("fallback list does not fit")
        out = {}
        for line in buf.value.decode().splitlines():
            k, v = line.split()
            out[k] = int(v)
        return out


def copy(dst, dst_dev, src, src_dev, nbytes):
    """Synchronous copy between host (-1) and device memories."""
    if lib().pa_nat_copy(dst, int(dst_dev), src, int(src_dev), int(nbytes)) != 0:
        raise RuntimeError(_err())

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.pa_nat_executor_free(self._h)
