"""ctypes binding of the native C++ runtime (``lib/libpaddle_amd_runtime.so``).

Components (see csrc/runtime/*.cc): RecordIO writer/scanner, LoDTensor stream IO,
buddy allocator (+ torch pluggable-allocator hooks), blocking record queue with
C++ RecordIO reader threads, DAG scheduler, profiler event buffers.
"""
from __future__ import annotations

import collections
import ctypes
import os
import threading

import numpy as np

from . import _build

_lib = None
_lock = threading.Lock()
P, I, SZ, U64P, I64P = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint64), \
    ctypes.POINTER(ctypes.c_int64)
NODE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_int, ctypes.c_void_p)

_SIGS = {
    "pa_rt_last_error": ([], ctypes.c_char_p),
    "pa_opt_create": ([ctypes.c_char_p, I, I, P, I, ctypes.c_char_p, I], P),
    "pa_opt_release": ([P], I),
    "pa_opt_update": ([P, I, P, I], I),
    "pa_opt_get_weights": ([P, ctypes.POINTER(ctypes.c_void_p)], I),
    "pa_opt_get_state": ([P, ctypes.POINTER(ctypes.c_char_p)], I),
    "pa_rio_writer_open": ([ctypes.c_char_p, I, I], P),
    "pa_rio_writer_write": ([P, ctypes.c_char_p, SZ], I),
    "pa_rio_writer_close": ([P], I),
    "pa_rio_scanner_open": ([ctypes.c_char_p], P),
    "pa_rio_scanner_next": ([P, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(SZ)], I),
    "pa_rio_scanner_close": ([P], None),
    "pa_ts_open": ([ctypes.c_char_p, I, I], P),
    "pa_ts_close": ([P], I),
    "pa_ts_write_lod_tensor": ([P, I, U64P, I64P, I, I, I64P, P, SZ], I),
    "pa_ts_read_header": ([P, ctypes.POINTER(I), U64P, I64P, I, I, ctypes.POINTER(I), ctypes.POINTER(I), I64P, I,
                           ctypes.POINTER(SZ), ctypes.POINTER(ctypes.c_int * 32)], I),
    "pa_ts_read_data": ([P, P, SZ], I),
    "pa_buddy_create": ([I, SZ, I], P),
    "pa_buddy_destroy": ([P], None),
    "pa_buddy_alloc": ([P, SZ], P),
    "pa_buddy_free": ([P, P], I),
    "pa_buddy_stats": ([P, ctypes.POINTER(SZ), ctypes.POINTER(SZ), ctypes.POINTER(SZ), ctypes.POINTER(SZ)], None),
    "pa_torch_set_chunk": ([SZ], None),
    "pa_torch_deferred_frees": ([], SZ),
    "pa_torch_stats": ([I, ctypes.POINTER(SZ), ctypes.POINTER(SZ), ctypes.POINTER(SZ)], None),
    "pa_bq_create": ([SZ], P),
    "pa_bq_push": ([P, ctypes.c_char_p, SZ], I),
    "pa_bq_pop": ([P, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(SZ), I], I),
    "pa_bq_size": ([P], SZ),
    "pa_bq_close": ([P], None),
    "pa_bq_destroy": ([P], None),
    "pa_rt_free": ([P], None),
    "pa_dc_get": ([I], P),
    "pa_dc_stream": ([P, I], P),
    "pa_dc_device": ([P], I),
    "pa_dc_event_acquire": ([P], P),
    "pa_dc_event_release": ([P, P], None),
    "pa_dc_stream_wait": ([P, I, I], I),
    "pa_dc_wait": ([P], I),
    "pa_dc_events_created": ([P], ctypes.c_long),
    "pa_dc_events_pooled": ([P], ctypes.c_long),
    "pa_dbr_create": ([I, SZ, I], P),
    "pa_dbr_push": ([P, I, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_int64)], I),
    "pa_dbr_close": ([P], None),
    "pa_dbr_next": ([P, ctypes.POINTER(ctypes.c_int64), I, I], I),
    "pa_dbr_consume": ([P, I, ctypes.POINTER(ctypes.c_void_p), P], I),
    "pa_dbr_queued": ([P], SZ),
    "pa_dbr_reset": ([P], None),
    "pa_dbr_destroy": ([P], None),
    "pa_bq_start_recordio_readers": ([P, ctypes.POINTER(ctypes.c_char_p), I, I, I], I),
    "pa_dag_run": ([I, ctypes.POINTER(I), ctypes.POINTER(I), ctypes.POINTER(I), I, NODE_FN, P], I),
    "pa_prof_enable": ([I], None),
    "pa_prof_push": ([ctypes.c_char_p], None),
    "pa_prof_pop": ([], None),
    "pa_prof_reset": ([], None),
    "pa_prof_dump": ([ctypes.c_char_p], ctypes.c_long),
}


def lib():
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(_build.RUNTIME_LIB):
                _build.build_runtime()
            import torch  # noqa: F401  (HIP runtime loaded first)

            L = ctypes.CDLL(_build.RUNTIME_LIB, mode=ctypes.RTLD_GLOBAL)
            for n, (a, r) in _SIGS.items():
                f = getattr(L, n)
                f.argtypes = a
                f.restype = r
            _lib = L
    return _lib


def available():
    try:
        lib()
        return True
    except Exception:
        return False


def _err():
    return lib().pa_rt_last_error().decode()


# ------------------------------------------------------------------ RecordIO


class RecordIOWriter:
    def __init__(self, path, compressor=2, max_num_records=1000):
        self._h = lib().pa_rio_writer_open(path.encode(), int(compressor), int(max_num_records))
        if not self._h:
            raise IOError(_err())

    def write(self, record: bytes):
        if lib().pa_rio_writer_write(self._h, record, len(record)) != 0:
            raise IOError(_err())

    def close(self):
        if self._h:
            rc = lib().pa_rio_writer_close(self._h)
            self._h = None
            if rc != 0:
                raise IOError(_err())

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class RecordIOScanner:
    def __init__(self, path):
        self._h = lib().pa_rio_scanner_open(path.encode())
        if not self._h:
            raise IOError(_err())

    def __iter__(self):
        d, n = ctypes.c_void_p(), SZ()
        while True:
            rc = lib().pa_rio_scanner_next(self._h, ctypes.byref(d), ctypes.byref(n))
            if rc == 0:
                break
            if rc < 0:
                raise IOError(_err())
            yield ctypes.string_at(d.value, n.value)
        self.close()

    def close(self):
        if self._h:
            lib().pa_rio_scanner_close(self._h)
            self._h = None


# ------------------------------------------------------------------ LoDTensor streams

_ES = (ctypes.c_int * 32)(*([0] * 32))
for _k, _v in {0: 1, 1: 2, 2: 4, 3: 8, 4: 2, 5: 4, 6: 8, 19: 8, 20: 1, 21: 1, 22: 2}.items():
    _ES[_k] = _v


def write_lod_tensors(path, tensors, append=False):
    """tensors: list of (numpy array, lod list-of-lists, vartype int)."""
    h = lib().pa_ts_open(path.encode(), 1, int(append))
    if not h:
        raise IOError(_err())
    try:
        for arr, lod, vt in tensors:
            arr = np.ascontiguousarray(arr)
            flat = np.asarray([x for lvl in lod for x in lvl], dtype=np.uint64)
            lens = np.asarray([len(l) for l in lod], dtype=np.int64)
            dims = np.asarray(arr.shape, dtype=np.int64)
            rc = lib().pa_ts_write_lod_tensor(
                h, len(lod), flat.ctypes.data_as(U64P), lens.ctypes.data_as(I64P), int(vt), arr.ndim,
                dims.ctypes.data_as(I64P), arr.ctypes.data_as(P), arr.nbytes)
            if rc != 0:
                raise IOError(_err())
    finally:
        lib().pa_ts_close(h)


_NPT = {0: np.bool_, 1: np.int16, 2: np.int32, 3: np.int64, 4: np.float16, 5: np.float32, 6: np.float64,
        19: np.uint64, 20: np.uint8, 21: np.int8, 22: np.uint16}


def read_lod_tensors(path, max_lod=1 << 20):
    """Returns list of (numpy array, lod, vartype).  bf16 (22) comes back as uint16 bits."""
    h = lib().pa_ts_open(path.encode(), 0, 0)
    if not h:
        raise IOError(_err())
    out = []
    fsize = os.path.getsize(path)
    try:
        lod_flat = (ctypes.c_uint64 * max_lod)()
        lod_lens = (ctypes.c_int64 * 16)()
        dims = (ctypes.c_int64 * 16)()
        while True:
            ll, dt, nd, nb = I(), I(), I(), SZ()
            rc = lib().pa_ts_read_header(h, ctypes.byref(ll), lod_flat, lod_lens, 16, max_lod, ctypes.byref(dt),
                                         ctypes.byref(nd), dims, 16, ctypes.byref(nb), ctypes.byref(_ES))
            if rc == 0:
                break
            if rc < 0:
                raise IOError(_err())
            lod, p = [], 0
            for i in range(ll.value):
                lod.append([int(lod_flat[p + k]) for k in range(lod_lens[i])])
                p += lod_lens[i]
            shape = [dims[i] for i in range(nd.value)]
            if dt.value not in _NPT:
                raise IOError(f"unsupported tensor dtype {dt.value} in {path}")
            if nb.value > fsize:
                raise IOError(f"tensor of {nb.value} bytes declared in a {fsize}-byte file {path}")
            arr = np.empty(shape, dtype=_NPT[dt.value])
            if lib().pa_ts_read_data(h, arr.ctypes.data_as(P), nb.value) != 0:
                raise IOError("truncated tensor data")
            out.append((arr, lod, dt.value))
    finally:
        lib().pa_ts_close(h)
    return out


# ------------------------------------------------------------------ allocator


class BuddyAllocator:
    def __init__(self, device=-1, chunk_bytes=1 << 30, init_mem=False):
        self._h = lib().pa_buddy_create(int(device), int(chunk_bytes), int(init_mem))

    def alloc(self, n):
        p = lib().pa_buddy_alloc(self._h, int(n))
        if not p:
            raise MemoryError(_err())
        return p

    def free(self, p):
        if lib().pa_buddy_free(self._h, p) != 0:
            raise ValueError(_err())

    def stats(self):
        u, r, pk, na = SZ(), SZ(), SZ(), SZ()
        lib().pa_buddy_stats(self._h, ctypes.byref(u), ctypes.byref(r), ctypes.byref(pk), ctypes.byref(na))
        return {"used": u.value, "reserved": r.value, "peak": pk.value, "arenas": na.value}

    def __del__(self):
        try:
            if self._h:
                lib().pa_buddy_destroy(self._h)
        except Exception:
            pass


def use_buddy_allocator_for_torch(chunk_bytes=4 << 30):
    """Route torch's HIP allocations through the native buddy allocator
    (FLAGS_allocator_strategy=buddy).  Must run before the first GPU allocation."""
    import torch

    lib().pa_torch_set_chunk(int(chunk_bytes))
    alloc = torch.cuda.memory.CUDAPluggableAllocator(_build.RUNTIME_LIB, "pa_torch_malloc", "pa_torch_free")
    # Tensor.record_stream: frees of blocks used on other streams wait for an event
    # on each of them (without the hook torch's pluggable path ignores record_stream)
    rs = ctypes.cast(getattr(ctypes.CDLL(_build.RUNTIME_LIB), "pa_torch_record_stream"), ctypes.c_void_p).value
    alloc._allocator.set_record_stream_fn(rs)
    torch.cuda.memory.change_current_allocator(alloc)
    global _BUDDY_ACTIVE
    _BUDDY_ACTIVE = True


_BUDDY_ACTIVE = False


def buddy_active():
    """True when torch's device allocations come from the buddy allocator."""
    return _BUDDY_ACTIVE


def torch_deferred_frees():
    """Blocks freed by torch but still waiting for another stream (record_stream)."""
    return int(lib().pa_torch_deferred_frees())


def torch_allocator_stats(device=0):
    """(used, reserved, peak) bytes of the buddy allocator behind torch on ``device``
    (all zero when it is not installed).  ``used`` includes blocks whose release is
    still waiting for their stream."""
    u, r, pk = SZ(), SZ(), SZ()
    lib().pa_torch_stats(int(device), ctypes.byref(u), ctypes.byref(r), ctypes.byref(pk))
    return {"used": u.value, "reserved": r.value, "peak": pk.value}


# ------------------------------------------------------------------ blocking queue


class BlockingQueue:
    def __init__(self, capacity):
        self._h = lib().pa_bq_create(int(capacity))

    def push(self, data: bytes) -> bool:
        return lib().pa_bq_push(self._h, data, len(data)) == 0

    def pop(self, timeout_ms=-1):
        p, n = ctypes.c_void_p(), SZ()
        rc = lib().pa_bq_pop(self._h, ctypes.byref(p), ctypes.byref(n), int(timeout_ms))
        if rc == 0:
            return None
        if rc < 0:
            raise TimeoutError("BlockingQueue.pop timed out")
        try:
            return ctypes.string_at(p.value, n.value)
        finally:
            lib().pa_rt_free(p)

    def size(self):
        return lib().pa_bq_size(self._h)

    def close(self):
        lib().pa_bq_close(self._h)

    def start_recordio_readers(self, paths, nthreads=2, passes=1):
        arr = (ctypes.c_char_p * len(paths))(*[p.encode() for p in paths])
        self._paths_keep = arr
        lib().pa_bq_start_recordio_readers(self._h, arr, len(paths), int(nthreads), int(passes))

    def __del__(self):
        try:
            if self._h:
                lib().pa_bq_destroy(self._h)
        except Exception:
            pass


# ------------------------------------------------------------------ double-buffer reader


class DoubleBufferReader:
    """Native py_reader pipeline (csrc/runtime/reader.cc; reference
    operators/reader/buffered_reader.cc, lod_tensor_blocking_queue.h): ``push``
    stages a batch of numpy arrays in pinned host memory (blocks while
    ``capacity`` batches wait), a C++ thread copies batches to ``nslots`` device
    slots on its own HIP stream, and ``next`` hands the oldest one to the current
    torch stream (event wait + device-to-device copy, no host sync).  ``device``
    None = host mode (CPU tensors, same queue logic)."""

    def __init__(self, capacity=2, nslots=2, device=None):
        import torch

        self.device = device
        self._torch = torch
        dev = -1 if device is None else int(torch.device(device).index or 0)
        self._h = lib().pa_dbr_create(int(nslots), int(capacity), dev)
        if not self._h:
            raise RuntimeError(_err())
        self._meta = collections.deque()  # (shapes, dtypes) per pushed batch, FIFO
        self._mu = threading.Lock()

    def push(self, arrays) -> bool:
        import numpy as np

        arrs = [np.ascontiguousarray(a) for a in arrays]
        n = len(arrs)
        ptrs = (ctypes.c_void_p * n)(*[a.ctypes.data for a in arrs])
        nbytes = (ctypes.c_int64 * n)(*[a.nbytes for a in arrs])
        with self._mu:  # meta order == queue order (one producer at a time)
            self._meta.append(([a.shape for a in arrs], [a.dtype for a in arrs]))
            rc = lib().pa_dbr_push(self._h, n, ptrs, nbytes)
            if rc != 0:
                self._meta.pop()
        if rc == -2:
            raise MemoryError(_err())
        return rc == 0

    def close(self):
        lib().pa_dbr_close(self._h)

    def next(self, timeout_ms=-1):
        """The next batch as a list of tensors (on ``device``), or None at EOF."""
        import numpy as np

        torch = self._torch
        nb = (ctypes.c_int64 * 64)()
        s = lib().pa_dbr_next(self._h, nb, 64, int(timeout_ms))
        if s == -1:
            return None
        if s == -2:
            raise TimeoutError("DoubleBufferReader.next timed out")
        if s < 0:
            raise RuntimeError(_err())
        shapes, dtypes = self._meta.popleft()
        outs = [torch.empty(tuple(sh), dtype=torch.from_numpy(np.empty(0, dt)).dtype,
                            device=self.device if self.device is not None else "cpu")
                for sh, dt in zip(shapes, dtypes)]
        dst = (ctypes.c_void_p * len(outs))(*[o.data_ptr() if o.numel() else None for o in outs])
        stream = torch.cuda.current_stream(self.device).cuda_stream if self.device is not None else None
        if lib().pa_dbr_consume(self._h, s, dst, stream) != 0:
            raise RuntimeError(_err())
        return outs

    def queued(self):
        return lib().pa_dbr_queued(self._h)

    def reset(self):
        lib().pa_dbr_reset(self._h)
        self._meta.clear()

    def __del__(self):
        try:
            if self._h:
                lib().pa_dbr_destroy(self._h)
                self._h = None
        except Exception:
            pass


# ------------------------------------------------------------------ DAG scheduler


def dag_run(n, edges, fn, nthreads=4):
    """Run ``fn(i)`` for every node i of a DAG (edges: list of (u, v) meaning u before v)
    on a C++ thread pool; the first exception is re-raised after in-flight nodes finish."""
    succ = [[] for _ in range(n)]
    indeg = [0] * n
    for u, v in edges:
        succ[u].append(v)
        indeg[v] += 1
    off = [0]
    flat = []
    for s in succ:
        flat += s
        off.append(len(flat))
    err = []

    def cb(node, _user):
        try:
            fn(node)
            return 0
        except BaseException as e:  # noqa: BLE001
            err.append(e)
            return 1

    c_cb = NODE_FN(cb)
    A = lambda xs: (ctypes.c_int * max(1, len(xs)))(*xs)  # noqa: E731
    rc = lib().pa_dag_run(n, A(indeg), A(off), A(flat), int(nthreads), c_cb, None)
    if err:
        raise err[0]
    if rc != 0:
        raise RuntimeError(_err())


# ------------------------------------------------------------------ profiler buffers


class NativeProfiler:
    @staticmethod
    def enable(on=True):
        lib().pa_prof_enable(int(on))

    @staticmethod
    def push(name):
        lib().pa_prof_push(name.encode())

    @staticmethod
    def pop():
        lib().pa_prof_pop()

    @staticmethod
    def reset():
        lib().pa_prof_reset()

    @staticmethod
    def dump(path):
        return lib().pa_prof_dump(path.encode())
