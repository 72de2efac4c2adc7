"""Strict-native mode: prove that a model or a test stayed on the framework's own
HIP kernels.

Reference behaviour: ``OperatorWithKernel::RunImpl`` looks up the kernel
registered for the expected ``OpKernelType`` and throws when there is none
(paddle/fluid/framework/operator.cc:665-685) -- there is no silent detour through
another library.  Here several layers *can* fall back to ATen (PyTorch-ROCm's own
kernels) for shapes or dtypes the HIP kernels do not cover; this module makes
every such detour visible and, under ``FLAGS_strict_native=1``, an error:

* :func:`region` brackets framework code (one Fluid op run, one eager-engine op,
  one tensor-API call, one reverse pass).  While the outermost region is open and
  counting is on (``FLAGS_strict_native=1`` or ``FLAGS_count_aten=1``), a
  ``TorchDispatchMode`` classifies every ATen call that touches a GPU tensor:
  allocation, view and metadata ops are free; anything else launches an ATen
  device kernel and is counted in :data:`ATEN_KERNELS` under
  ``"<region label>:<aten op>"`` -- or raises :class:`StrictNativeError` in strict
  mode.  The framework's HIP kernels are launched through raw pointers
  (``ops/_native.py``) and never pass through the dispatcher, so they are never
  counted.  Code outside every region (a test's own torch oracle) is not watched.
* :func:`fallback` is the explicit hook for code paths that know they are leaving
  the native kernels (e.g. an op branch for an unsupported dtype):
  :data:`FALLBACKS` counts them per site.

``reset()`` clears the counters; ``report()`` returns both as plain dicts.
"""
from __future__ import annotations

import contextlib
import os
import threading

import torch
from torch.utils._python_dispatch import TorchDispatchMode

ATEN_KERNELS: dict = {}   # "label:aten_op" -> ATen kernel launches on GPU tensors inside regions
NATIVE_OPS: dict = {}     # aten op -> calls executed on the framework's HIP kernels (ops/aten_native.py)
SYNCS: dict = {}          # region label -> device->host scalar reads (item() / float())
FALLBACKS: dict = {}      # site -> explicit fallback count
ATEN_SITES: dict = {}     # "label:aten_op" -> {"file:line" of the framework frame that issued it: count}
                          # (FLAGS_strict_trace=1: find the code behind each counted kernel)
NATIVE_SITES: dict = {}   # aten op -> {"file:line": count} of the calls run natively (FLAGS_strict_trace=1)
_TLS = threading.local()
# device types whose ATen kernels count (tests add "cpu" to exercise the watcher here)
WATCH_DEVICES = {"cuda"}


class StrictNativeError(RuntimeError):
    """An ATen device kernel (or an explicit fallback) ran inside a framework region
    under ``FLAGS_strict_native=1``."""


def strict() -> bool:
    return os.environ.get("FLAGS_strict_native", "0") not in ("0", "", "false", "False")


def counting() -> bool:
    return strict() or os.environ.get("FLAGS_count_aten", "0") not in ("0", "", "false", "False")


_CUDA = []


def inside() -> bool:
    """Already inside a framework region (nested framework code needs no region of
    its own: the outer one's dispatch mode is active)."""
    return bool(getattr(_TLS, "labels", None))


def watching() -> bool:
    """True when a region would push the dispatch mode (native dispatch or counting)."""
    return native_dispatch() or counting()


def native_dispatch() -> bool:
    """Route ATen pointwise / cast / fill / reduction ops issued inside framework
    regions onto the HIP kernels of ops/aten_native.py (default on with a GPU)."""
    if os.environ.get("FLAGS_native_dispatch", "1") in ("0", "false", "False"):
        return False
    if not _CUDA:
        _CUDA.append(torch.cuda.is_available())
    return _CUDA[0]


# ATen ops that launch no device kernel: allocation, views, metadata, stream bookkeeping
_FREE = {
    "empty", "empty_strided", "empty_like", "new_empty", "new_empty_strided", "resize_", "set_",
    "view", "_unsafe_view", "reshape", "as_strided", "t", "transpose", "permute", "expand", "expand_as",
    "squeeze", "unsqueeze", "select", "slice", "narrow", "split", "split_with_sizes", "unbind", "chunk",
    "detach", "alias", "lift_fresh", "view_as", "unflatten", "flatten", "diagonal", "movedim",
    "record_stream", "is_same_size", "_reshape_alias", "numpy_T", "real", "conj", "resolve_conj",
    "resolve_neg", "_conj", "_neg_view", "clone_view", "contiguous_view", "split_copy_view", "unfold",
    "is_pinned", "size", "stride", "dim", "sym_size", "sym_stride", "sym_numel", "sym_storage_offset",
    "_local_scalar_dense_view",
}


def _is_gpu(x):
    return isinstance(x, torch.Tensor) and x.device.type in WATCH_DEVICES


_META = {}  # OpOverload -> (op name, watched?)


def _label():
    labels = getattr(_TLS, "labels", None)
    return labels[-1] if labels else "?"


def _crosses_host(args, kwargs):
    """A copy with one side in host memory (H2D / D2H transfer)."""
    devs = set()
    for a in list(args) + list(kwargs.values()):
        if isinstance(a, torch.Tensor):
            devs.add(a.device.type)
    dev = kwargs.get("device")
    if dev is not None:
        devs.add(torch.device(dev).type)
    return "cpu" in devs and len(devs) > 1


def _touches_gpu(args, kwargs):
    dev = kwargs.get("device")
    if dev is not None and torch.device(dev).type in WATCH_DEVICES:
        return True  # factory op (zeros / full / empty ...) placed on the GPU
    for a in args:
        if _is_gpu(a):
            return True
        if isinstance(a, (list, tuple)) and any(_is_gpu(b) for b in a):
            return True
    for a in kwargs.values():
        if _is_gpu(a):
            return True
    return False


class _Watch(TorchDispatchMode):
    def __init__(self, native):
        super().__init__()
        self.native = native

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        meta = _META.get(func)
        if meta is None:
            ns = getattr(func, "namespace", "aten")
            nm = func._schema.name.split("::")[-1] if hasattr(func, "_schema") else str(func)
            meta = _META[func] = (nm, ns == "aten" and nm not in _FREE)
        name, watched = meta
        if watched and _touches_gpu(args, kwargs):
            if name in ("_to_copy", "copy_") and _crosses_host(args, kwargs):
                return func(*args, **kwargs)  # host <-> device transfer: a DMA copy, no kernel
            if name == "_local_scalar_dense":
                SYNCS[_label()] = SYNCS.get(_label(), 0) + 1  # device -> host read (a sync)
                return func(*args, **kwargs)
            nat = getattr(_TLS, "natives", None)
            if self.native and nat and nat[-1]:
                from ..ops import aten_native

                r = aten_native.try_native(func, args, kwargs)
                if r is not NotImplemented:
                    NATIVE_OPS[name] = NATIVE_OPS.get(name, 0) + 1
                    if os.environ.get("FLAGS_strict_trace", "0") not in ("0", ""):
                        d = NATIVE_SITES.setdefault(name, {})
                        site = _site()
                        d[site] = d.get(site, 0) + 1
                    return r
            # a contiguous() of an already contiguous tensor never reaches here;
            # clone / copy_ / _to_copy do launch a copy kernel and are counted
            labels = getattr(_TLS, "labels", None)
            key = f"{labels[-1] if labels else '?'}:{name}"
            ATEN_KERNELS[key] = ATEN_KERNELS.get(key, 0) + 1
            if os.environ.get("FLAGS_strict_trace", "0") not in ("0", ""):
                site = _site()
                d = ATEN_SITES.setdefault(key, {})
                d[site] = d.get(site, 0) + 1
            if strict():
                raise StrictNativeError(
                    f"FLAGS_strict_native: ATen kernel aten::{name} launched on a GPU tensor inside "
                    f"framework region '{labels[-1] if labels else '?'}' (no native kernel covers this call)")
        return func(*args, **kwargs)


_SKIP_SITES = (os.sep + os.path.join("utils", "strict.py"), os.sep + os.path.join("ops", "aten_native.py"))


def _site():
    """file:line of the innermost framework frame outside this module / the native
    dispatch layer (the code that issued the ATen call)."""
    import sys

    f = sys._getframe(2)
    while f is not None:
        fn = f.f_code.co_filename
        if "paddle_amd" in fn and not fn.endswith(_SKIP_SITES):
            return f"{fn[fn.rfind('paddle_amd'):]}:{f.f_lineno}"
        f = f.f_back
    return "?"


class region:
    """Bracket framework code; only the outermost region pushes the dispatch mode.
    ``native``: run covered ATen ops on the HIP kernels (else only count).  A plain
    class (not a generator context manager) and one reused mode object per thread:
    this is entered once per eager op."""

    __slots__ = ("label", "native", "mode")

    def __init__(self, label: str, native: bool = True):
        self.label, self.native, self.mode = label, native, None

    def __enter__(self):
        labels = getattr(_TLS, "labels", None)
        if labels is None:
            labels = _TLS.labels = []
            _TLS.natives = []
        outer = not labels
        labels.append(self.label)
        _TLS.natives.append(bool(self.native))  # the innermost region decides native execution
        if outer and (native_dispatch() or counting()):
            m = getattr(_TLS, "mode", None)
            nat = native_dispatch()
            if m is None or m.native != nat:
                m = _TLS.mode = _Watch(nat)
            m.__enter__()
            self.mode = m
        return self

    def __exit__(self, *exc):
        if self.mode is not None:
            self.mode.__exit__(None, None, None)
            self.mode = None
        _TLS.labels.pop()
        _TLS.natives.pop()
        return False


@contextlib.contextmanager
def unwatched():
    """Temporarily leave every region (e.g. a deliberate host-side reference path
    the caller accounts for itself)."""
    labels = getattr(_TLS, "labels", None)
    saved = list(labels) if labels else []
    nsaved = list(getattr(_TLS, "natives", []) or [])
    if labels:
        labels.clear()
        _TLS.natives.clear()
    try:
        from torch.utils._python_dispatch import _pop_mode_temporarily, _get_current_dispatch_mode

        if saved and isinstance(_get_current_dispatch_mode(), _Watch):
            with _pop_mode_temporarily():
                yield
        else:
            yield
    finally:
        if labels is not None:
            labels[:] = saved
            _TLS.natives[:] = nsaved


def fallback(site: str, on_gpu: bool = True):
    """Record an explicit fallback off the native kernels at ``site``; raises in strict mode."""
    FALLBACKS[site] = FALLBACKS.get(site, 0) + 1
    if on_gpu and strict():
        raise StrictNativeError(f"FLAGS_strict_native: '{site}' left the native kernels")


def reset():
    ATEN_KERNELS.clear()
    ATEN_SITES.clear()
    NATIVE_SITES.clear()
    FALLBACKS.clear()
    NATIVE_OPS.clear()
    SYNCS.clear()


def report() -> dict:
    rep = {"aten_kernels": dict(ATEN_KERNELS), "fallbacks": dict(FALLBACKS), "native_ops": dict(NATIVE_OPS),
           "syncs": dict(SYNCS)}
    if ATEN_SITES:
        rep["aten_sites"] = {k: dict(v) for k, v in ATEN_SITES.items()}
    if NATIVE_SITES:
        rep["native_sites"] = {k: dict(v) for k, v in NATIVE_SITES.items()}
    return rep
