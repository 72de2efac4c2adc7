"""Platform services (reference paddle/fluid/platform: init.cc InitDevices / InitP2P,
gpu_info.cc memory queries, enforce.h, and the glog VLOG / GLOG_v verbosity used
throughout the C++ core).

* ``vlog(level, msg)``: printed to stderr when ``GLOG_v`` (or ``FLAGS_v``) >= level;
  the executor logs every op at level 3 and memory statistics at level 1 (or every
  run when ``FLAGS_log_memory_stats=1``);
* ``enforce(cond, msg)`` / ``EnforceError`` (the kernel library's HIP errors carry
  the error name, ``ops._native.EnforceError``);
* ``init_p2p(devices)`` enables peer access between every pair of the node's GPUs
  that supports it (xGMI), ``memcpy_peer(dst, src)`` copies across devices without
  staging through the host;
* ``device_memory_info(dev)`` / ``memory_stats(dev)``;
* ``DeviceContextPool.instance().get(place)`` -> ``DeviceContext`` (reference
  platform/device_context.h:39-179): per HIP device a compute, a high-priority
  communication and an auxiliary stream plus an event pool, owned by the native
  runtime (csrc/runtime/device_context.cc) and exposed to torch as external
  streams; the ParallelExecutor's and the sharded optimizer's collective streams
  and the overlapped optimizer update run on them.
"""
from __future__ import annotations

import ctypes
import os
import sys
import time

import torch

from .ops import _native as N
from .ops._native import EnforceError  # noqa: F401

_V = int(os.environ.get("GLOG_v", os.environ.get("FLAGS_v", "0")) or 0)


def vlog_level() -> int:
    return _V


def set_vlog_level(v: int):
    global _V
    _V = int(v)


def vlog(level: int, msg: str):
    if _V >= level:
        t = time.strftime("%H:%M:%S")
        sys.stderr.write(f"I{t} {os.getpid()} paddle_amd] {msg}\n")


def enforce(cond, msg="enforce failed", *args):
    if not cond:
        raise EnforceError.__bases__[0](msg % args if args else msg)


def device_count() -> int:
    n = ctypes.c_int(0)
    N.check(N.lib().pa_device_count(ctypes.byref(n)), "pa_device_count")
    return n.value


def init_p2p(devices=None):
    """Enable peer access for every ordered pair of ``devices`` that can access
    each other (reference platform/init.cc InitP2P).  Returns the enabled pairs."""
    lib = N.lib()
    devs = list(range(device_count())) if devices is None else list(devices)
    pairs = []
    for a in devs:
        for b in devs:
            if a == b:
                continue
            can = ctypes.c_int(0)
            N.check(lib.pa_can_access_peer(a, b, ctypes.byref(can)), "pa_can_access_peer")
            if can.value:
                N.check(lib.pa_enable_peer_access(a, b), "pa_enable_peer_access")
                pairs.append((a, b))
    vlog(1, f"init_p2p: {len(pairs)} peer pairs enabled over devices {devs}")
    return pairs


def memcpy_peer(dst: torch.Tensor, src: torch.Tensor):
    """dst[...] = src[...] across devices on the current stream (hipMemcpyPeerAsync)."""
    enforce(dst.is_cuda and src.is_cuda, "memcpy_peer: device tensors")
    enforce(dst.is_contiguous() and src.is_contiguous() and dst.dtype == src.dtype
            and dst.numel() == src.numel(), "memcpy_peer: matching contiguous tensors")
    N.call("pa_memcpy_peer_async", N.ptr(dst), dst.device.index, N.ptr(src), src.device.index,
           src.numel() * src.element_size(), N.stream())
    return dst


def device_memory_info(dev=0):
    """(free, total) bytes of HBM on ``dev`` (hipMemGetInfo)."""
    f, t = ctypes.c_size_t(0), ctypes.c_size_t(0)
    N.check(N.lib().pa_mem_info(int(dev), ctypes.byref(f), ctypes.byref(t)), "pa_mem_info")
    return f.value, t.value


def memory_stats(dev=0):
    """Allocator + device view of memory (reference: the memory-usage VLOGs of
    buddy_allocator.cc / gpu_info.cc): ``allocated`` / ``reserved`` / ``peak`` bytes
    from whichever allocator backs torch (the buddy allocator's peak is the sum of
    its per-stream pool peaks, an upper bound), plus the device's free / total."""
    from . import runtime

    out = {}
    if runtime.buddy_active():
        st = runtime.torch_allocator_stats(dev)
        out.update(allocated=st["used"], reserved=st["reserved"], peak=st["peak"], allocator="buddy")
    else:
        out.update(allocated=torch.cuda.memory_allocated(dev), reserved=torch.cuda.memory_reserved(dev),
                   peak=torch.cuda.max_memory_allocated(dev), allocator="torch_caching")
    free, total = device_memory_info(dev)
    out.update(device_free=free, device_total=total)
    return out


def memory_allocated(dev=0):
    return memory_stats(dev)["allocated"]


def max_memory_allocated(dev=0):
    return memory_stats(dev)["peak"]


def log_memory(tag, dev=0):
    if torch.cuda.is_available():
        st = memory_stats(dev)
        vlog(0 if os.environ.get("FLAGS_log_memory_stats") == "1" else 1,
             f"memory[{tag}] " + " ".join(f"{k}={v / 2**30:.2f}GiB" if isinstance(v, int) else f"{k}={v}"
                                          for k, v in st.items()))


# ------------------------------------------------------------------ device contexts
class DeviceContext:
    """One HIP device's streams (compute / comm / aux) and event pool."""

    COMPUTE, COMM, AUX = 0, 1, 2

    def __init__(self, device):
        from . import runtime

        self._rt = runtime.lib()
        self.device = torch.device("cuda", int(device))
        self._h = self._rt.pa_dc_get(int(self.device.index))
        if not self._h:
            raise RuntimeError(runtime._err())
        self._streams = {}

    def _stream(self, which):
        s = self._streams.get(which)
        if s is None:
            ptr = self._rt.pa_dc_stream(self._h, which)
            s = self._streams[which] = torch.cuda.ExternalStream(ptr, device=self.device)
        return s

    @property
    def stream(self):
        return self._stream(self.COMPUTE)

    @property
    def comm_stream(self):
        return self._stream(self.COMM)

    @property
    def aux_stream(self):
        return self._stream(self.AUX)

    def stream_wait(self, waiter, other):
        """``waiter`` stream waits on the device for the work queued on ``other``."""
        if self._rt.pa_dc_stream_wait(self._h, int(waiter), int(other)) != 0:
            raise RuntimeError("DeviceContext.stream_wait failed")

    def wait(self):
        """DeviceContext::Wait: block the host until every stream drained."""
        if self._rt.pa_dc_wait(self._h) != 0:
            raise RuntimeError("DeviceContext.wait failed")

    def event_pool_stats(self):
        return {"created": int(self._rt.pa_dc_events_created(self._h)),
                "pooled": int(self._rt.pa_dc_events_pooled(self._h))}


class DeviceContextPool:
    """Per-place device contexts (DeviceContextPool::Get); CPU places have none."""

    _inst = None

    def __init__(self):
        self._ctx = {}

    @classmethod
    def instance(cls):
        if cls._inst is None:
            cls._inst = cls()
        return cls._inst

    def get(self, place):
        if isinstance(place, torch.device):
            dev = place
        elif hasattr(place, "torch_device"):
            dev = place.torch_device()
        else:
            dev = torch.device(place)
        if dev.type != "cuda":
            return None
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        c = self._ctx.get(idx)
        if c is None:
            c = self._ctx[idx] = DeviceContext(idx)
        return c


def device_context(place):
    """The DeviceContext of ``place`` (None for CPU, or without the runtime library)."""
    try:
        return DeviceContextPool.instance().get(place)
    except (OSError, RuntimeError):
        return None
