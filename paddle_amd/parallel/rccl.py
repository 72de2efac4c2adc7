"""Framework-owned RCCL communicators (``csrc/runtime/rccl_comm.cc``).

Reference: platform/nccl_helper.h:49-123 -- ``NCCLGroupGuard`` (process-wide mutex
around ncclGroupStart/End) and ``NCCLContextMap`` (one communicator per place,
``InitRank`` with rank = trainer_id * ngpu + gpu_id) -- and
operators/gen_nccl_id_op.cc:54-110 (trainer 0 generates the ncclUniqueId and sends
it to the others over RPC).

MI355X-first: one process per GPU, so :class:`CommContextMap` maps a process group
(tuple of global ranks) to ONE :class:`Communicator` on this process's device.  The
unique id of each communicator is created by the group's first rank and published
in the job's TCP key-value store under a per-group, per-generation key (the
``gen_nccl_id`` role, without an extra RPC server).  Collectives are enqueued on
the caller's HIP stream (torch's current stream by default, or the DeviceContext
comm stream), so they order with the kernels that produced their inputs without a
host synchronisation, exactly like the framework's own kernels.

These communicators ARE the GPU communication layer: :mod:`paddle_amd.parallel.comm`
routes every collective on contiguous device tensors -- all-reduce, reduce-scatter,
all-gather, broadcast, the expert-parallel all-to-all (grouped ncclSend/ncclRecv)
and the pipeline's point-to-point exchanges -- through them whenever librccl loads
(``FLAGS_comm_backend`` = ``auto``, the default, or ``pa_rccl``).
``FLAGS_comm_backend=torch`` keeps ``torch.distributed``'s ProcessGroupNCCL; gloo /
host tensors always use ``torch.distributed``.

Failure handling: :meth:`CommContextMap.check_health` polls every communicator's
asynchronous error (a peer died or timed out) and aborts ALL of them
(``ncclCommAbort``) before raising, so no rank stays blocked inside a collective;
the elastic watchdog calls it (``distributed/elastic.py``).
"""
from __future__ import annotations

import contextlib
import ctypes
import math
import os
import threading

import torch

from .. import runtime as _rt

# ncclDataType_t / ncclRedOp_t values (rccl.h)
_DT = {torch.int8: 0, torch.uint8: 1, torch.int32: 2, torch.int64: 4, torch.float16: 6, torch.float32: 7,
       torch.float64: 8, torch.bfloat16: 9}
_OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}

_lock = threading.Lock()
_sigs_ready = [False]


def _lib():
    L = _rt.lib()
    if not _sigs_ready[0]:
        P, I, S = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        L.pa_rccl_last_error.restype = ctypes.c_char_p
        L.pa_rccl_unique_id.argtypes = [ctypes.c_char_p]
        L.pa_rccl_comm_init.argtypes = [ctypes.c_char_p, I, I, I, ctypes.POINTER(P)]
        L.pa_rccl_comm_destroy.argtypes = [P, I]
        L.pa_rccl_async_error.argtypes = [P]
        L.pa_rccl_all_reduce.argtypes = [P, P, S, I, I, P, P]
        L.pa_rccl_reduce_scatter.argtypes = [P, P, S, I, I, P, P]
        L.pa_rccl_all_gather.argtypes = [P, P, S, I, P, P]
        L.pa_rccl_broadcast.argtypes = [P, P, S, I, I, P, P]
        L.pa_rccl_send.argtypes = [P, S, I, I, P, P]
        L.pa_rccl_recv.argtypes = [P, S, I, I, P, P]
        SP = ctypes.POINTER(ctypes.c_size_t)
        L.pa_rccl_all_to_all.argtypes = [P, P, SP, SP, SP, SP, I, I, S, P, P]
        _sigs_ready[0] = True
    return L


class RcclError(RuntimeError):
    pass


class RcclUnavailable(RcclError):
    """Raised on EVERY rank of a group when any of its ranks cannot create its
    communicator (the verdict is agreed through the store before ncclCommInitRank)."""


def _local_ready(device: int) -> bool:
    """What this rank can check alone before joining a clique: librccl loads and (for a
    device communicator) the device index exists."""
    if not available():
        return False
    if device < 0:
        return True
    try:
        return 0 <= device < torch.cuda.device_count()
    except Exception:
        return False


def agree(store, key: str, world: int, rank: int, ok: bool, timeout_s: float = 300.0) -> list:
    """Every rank publishes ``ok`` under ``key`` and reads everyone's: returns the
    (group-local) ranks that reported failure -- the same list on every rank."""
    import datetime

    store.set(f"{key}/ready/{rank}", b"1" if ok else b"0")
    keys = [f"{key}/ready/{r}" for r in range(world)]
    store.wait(keys, datetime.timedelta(seconds=timeout_s))
    return [r for r, k in enumerate(keys) if bytes(store.get(k)) != b"1"]


def _check(rc, what):
    if rc != 0:
        raise RcclError(f"{what}: {_lib().pa_rccl_last_error().decode()}")


def available() -> bool:
    try:
        return bool(_lib().pa_rccl_available())
    except Exception:
        return False


def unique_id() -> bytes:
    buf = ctypes.create_string_buffer(128)
    _check(_lib().pa_rccl_unique_id(buf), "ncclGetUniqueId")
    return buf.raw


def _stream(stream, device=0):
    if device < 0:
        return ctypes.c_void_p()  # host communicator (fake library): no stream
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


class Communicator:
    """One RCCL communicator: ``world`` ranks, this process is ``rank``, on ``device``.

    ``uid``: the clique's 128-byte unique id (the same bytes on every rank); use
    :meth:`rendezvous` to create it on rank 0 and distribute it through a store.
    ``device`` < 0: host buffers (a multi-rank CPU test against a C-ABI fake)."""

    def __init__(self, uid: bytes, world: int, rank: int, device: int):
        if len(uid) != 128:
            raise ValueError("RCCL unique id must be 128 bytes")
        self.world, self.rank, self.device = int(world), int(rank), int(device)
        h = ctypes.c_void_p()
        _check(_lib().pa_rccl_comm_init(uid, self.world, self.rank, self.device, ctypes.byref(h)),
               "ncclCommInitRank")
        self._h = h

    @classmethod
    def rendezvous(cls, store, key: str, world: int, rank: int, device: int, timeout_s: float = 300.0):
        """gen_nccl_id: rank 0 publishes a fresh unique id under ``key``, every rank
        reads it from the store (blocking) and joins the clique."""
        if rank == 0:
            store.set(key, unique_id())
        store.wait([key], __import__("datetime").timedelta(seconds=timeout_s))
        uid = store.get(key)
        return cls(bytes(uid), world, rank, device)

    # ------------------------------------------------------------------ collectives
    def _args(self, t):
        if t.is_cuda != (self.device >= 0) or t.dtype not in _DT or not t.is_contiguous():
            raise RcclError(f"RCCL operand must be a contiguous {'device' if self.device >= 0 else 'host'} "
                            f"tensor of a supported dtype ({t.dtype}, {t.device})")
        return ctypes.c_void_p(t.data_ptr()), _DT[t.dtype]

    def _st(self, stream):
        return _stream(stream, self.device)

    def all_reduce(self, t, op="sum", stream=None):
        p, dt = self._args(t)
        _check(_lib().pa_rccl_all_reduce(p, p, t.numel(), dt, _OPS[op], self._h, self._st(stream)), "ncclAllReduce")

    def reduce_scatter(self, out, inp, op="sum", stream=None):
        po, dt = self._args(out)
        pi, _ = self._args(inp)
        if inp.numel() != out.numel() * self.world or inp.dtype != out.dtype:
            raise RcclError("reduce_scatter: input must hold world x output elements of the same dtype")
        _check(_lib().pa_rccl_reduce_scatter(pi, po, out.numel(), dt, _OPS[op], self._h, self._st(stream)),
               "ncclReduceScatter")

    def all_gather(self, out, inp, stream=None):
        po, dt = self._args(out)
        pi, _ = self._args(inp)
        if out.numel() != inp.numel() * self.world or inp.dtype != out.dtype:
            raise RcclError("all_gather: output must hold world x input elements of the same dtype")
        _check(_lib().pa_rccl_all_gather(pi, po, inp.numel(), dt, self._h, self._st(stream)), "ncclAllGather")

    def broadcast(self, t, root=0, stream=None):
        p, dt = self._args(t)
        _check(_lib().pa_rccl_broadcast(p, p, t.numel(), dt, int(root), self._h, self._st(stream)),
               "ncclBroadcast")

    def send(self, t, peer, stream=None):
        p, dt = self._args(t)
        _check(_lib().pa_rccl_send(p, t.numel(), dt, int(peer), self._h, self._st(stream)), "ncclSend")

    def recv(self, t, peer, stream=None):
        p, dt = self._args(t)
        _check(_lib().pa_rccl_recv(p, t.numel(), dt, int(peer), self._h, self._st(stream)), "ncclRecv")

    def all_to_all(self, out, inp, out_splits=None, in_splits=None, stream=None):
        """Rows of ``inp`` split by ``in_splits`` (one chunk per peer, rank order) are
        exchanged; ``out`` receives ``out_splits`` rows from each peer.  Equal splits
        when None.  One fused ncclSend/ncclRecv group (csrc pa_rccl_all_to_all)."""
        po, dt = self._args(out)
        pi, _ = self._args(inp)
        W = self.world
        if out.dtype != inp.dtype or out.shape[1:] != inp.shape[1:]:
            raise RcclError("all_to_all: input and output rows must match in dtype and shape")
        row = math.prod(inp.shape[1:])  # 1 for 1-D; works for zero-row sends
        ins = list(in_splits) if in_splits is not None else [inp.shape[0] // W] * W
        outs = list(out_splits) if out_splits is not None else [out.shape[0] // W] * W
        if len(ins) != W or len(outs) != W or sum(ins) != inp.shape[0] or sum(outs) != out.shape[0]:
            raise RcclError("all_to_all: splits must have one entry per rank and cover the rows")
        arr = ctypes.c_size_t * W
        sc = arr(*[n * row for n in ins])
        rc_ = arr(*[n * row for n in outs])
        sd = arr(*[sum(ins[:p]) * row for p in range(W)])
        rd = arr(*[sum(outs[:p]) * row for p in range(W)])
        _check(_lib().pa_rccl_all_to_all(pi, po, sc, sd, rc_, rd, W, dt, inp.element_size(), self._h,
                                         self._st(stream)), "ncclSend/ncclRecv all_to_all")

    def check_async(self):
        """Raise if the communicator hit an asynchronous error (a peer failed)."""
        _check(_lib().pa_rccl_async_error(self._h), "communicator")

    def destroy(self, abort=False):
        if getattr(self, "_h", None) is not None and self._h.value:
            _check(_lib().pa_rccl_comm_destroy(self._h, int(abort)), "ncclCommDestroy")
            self._h = ctypes.c_void_p()


@contextlib.contextmanager
def group_guard():
    """NCCLGroupGuard: the collectives issued inside launch as one fused group
    (ncclGroupStart/End, serialised across host threads)."""
    _check(_lib().pa_rccl_group_start(), "ncclGroupStart")
    try:
        yield
    finally:
        _check(_lib().pa_rccl_group_end(), "ncclGroupEnd")


class CommContextMap:
    """NCCLContextMap: process group (global ranks) -> this process's communicator."""

    def __init__(self, store=None):
        self._store = store
        self._comms = {}
        self._gen = {}

    def _default_store(self):
        if self._store is None:
            import torch.distributed as dist

            self._store = dist.distributed_c10d._get_default_store()
        return self._store

    def get(self, ranks, my_rank, device=None):
        """The communicator of the group with global ``ranks`` (sorted) for this process
        (global rank ``my_rank``); created on first use -- a collective over the group."""
        key = tuple(sorted(ranks))
        c = self._comms.get(key)
        if c is None:
            with _lock:
                c = self._comms.get(key)
                if c is None:
                    gen = self._gen.get(key, 0)
                    self._gen[key] = gen + 1
                    dev = torch.cuda.current_device() if device is None else device
                    name = f"pa_rccl/{'-'.join(map(str, key))}/{gen}"
                    store = self._default_store()
                    # collective go / no-go BEFORE ncclCommInitRank: a rank that cannot
                    # build its communicator (librccl missing, bad device) must not leave
                    # its peers blocked inside the init -- every rank sees the same
                    # verdict, so an ``auto`` fallback is taken by all ranks or by none
                    bad = agree(store, name, len(key), key.index(my_rank), _local_ready(dev))
                    if bad:
                        raise RcclUnavailable(f"framework RCCL unavailable on group ranks {bad} of {list(key)}")
                    c = Communicator.rendezvous(store, name, len(key), key.index(my_rank), dev)
                    self._comms[key] = c
        return c

    def destroy_all(self, abort=False):
        for c in self._comms.values():
            c.destroy(abort)
        self._comms.clear()

    def check_health(self):
        """Raise :class:`RcclError` if any communicator reports an asynchronous error;
        every communicator is aborted first (ncclCommAbort), so the collectives other
        host threads or streams are blocked in return instead of hanging."""
        for key, c in list(self._comms.items()):
            try:
                c.check_async()
            except RcclError as e:
                for other in self._comms.values():
                    try:
                        other.destroy(abort=True)
                    except RcclError:
                        pass
                self._comms.clear()
                raise RcclError(f"communicator of ranks {list(key)} failed ({e}); all communicators aborted") from e


_MAP = CommContextMap()


def context_map() -> CommContextMap:
    return _MAP


def enabled() -> bool:
    """Route device collectives through the framework communicators: ``auto`` (the
    default) whenever librccl loads, ``pa_rccl`` always, ``torch`` never."""
    mode = os.environ.get("FLAGS_comm_backend", "auto")
    if mode == "pa_rccl":
        return True
    if mode != "auto":
        return False
    if not _AUTO:
        _AUTO.append(torch.cuda.is_available() and available())
    return _AUTO[0]


_AUTO: list = []


def disable_auto(reason: str) -> None:
    """``auto`` mode: stop routing collectives through the framework communicators
    (the caller falls back to torch.distributed), with one warning."""
    import warnings

    warnings.warn(reason, RuntimeWarning, stacklevel=2)
    _AUTO[:] = [False]
