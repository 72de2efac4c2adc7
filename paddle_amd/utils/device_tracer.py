"""In-process kernel activity tracing on rocprofiler-sdk.

The reference's ``DeviceTracer`` (paddle/fluid/platform/device_tracer.h:45-92,
device_tracer.cc:98-121) buffers CUPTI kernel activity records inside the
training process and correlates them with the profiler's op annotations.  Here
the native tool library ``lib/libpaddle_amd_tracer.so`` (csrc/tracer/
device_tracer.cc) plays that role on rocprofiler-sdk: buffered KERNEL_DISPATCH
tracing with device start/end timestamps, a kernel-symbol table from code-object
tracing, and the framework's RecordEvent ranges pushed as external correlation
ids.

rocprofiler-sdk tools must be registered before the HIP runtime initialises, so
``install()`` has to run before the first device call of the process: importing
``paddle_amd`` with ``FLAGS_device_tracer=1`` (or ``PADDLE_AMD_DEVICE_TRACER=1``)
in the environment does it.  ``install()`` after HIP is up returns False and the
profiler keeps its HIP-event device track.
"""
from __future__ import annotations

import ctypes
import os
import shutil
import subprocess

_LIB = None
_STATE = {"installed": False, "error": None}


def _path():
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib", "libpaddle_amd_tracer.so")


def _load():
    global _LIB
    if _LIB is None:
        p = _path()
        if not os.path.exists(p):
            raise OSError(f"{p} not built (paddle_amd._build.build_tracer)")
        lib = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
        u64, i32, i64 = ctypes.c_uint64, ctypes.c_int32, ctypes.c_long
        lib.pa_tracer_register.restype = ctypes.c_int
        lib.pa_tracer_available.restype = ctypes.c_int
        lib.pa_tracer_enable.restype = ctypes.c_int
        lib.pa_tracer_disable.restype = ctypes.c_int
        lib.pa_tracer_flush.restype = ctypes.c_int
        lib.pa_tracer_now_ns.restype = u64
        lib.pa_tracer_push_range.argtypes = [u64]
        lib.pa_tracer_push_range.restype = ctypes.c_int
        lib.pa_tracer_pop_range.restype = ctypes.c_int
        lib.pa_tracer_count.restype = i64
        lib.pa_tracer_dropped.restype = u64
        lib.pa_tracer_get.argtypes = [i64, ctypes.POINTER(u64), ctypes.POINTER(i32), ctypes.c_char_p, ctypes.c_int]
        lib.pa_tracer_get.restype = ctypes.c_int
        lib.pa_tracer_last_error.restype = ctypes.c_int
        _LIB = lib
    return _LIB


def install() -> bool:
    """Load and register the tool (before any HIP call).  True when registered."""
    if _STATE["installed"]:
        return True
    try:
        rc = _load().pa_tracer_register()
    except OSError as e:
        _STATE["error"] = str(e)
        return False
    if rc != 0:
        _STATE["error"] = ("the HIP runtime was initialised before the tracer registered" if rc == -2
                           else f"rocprofiler_force_configure status {rc}")
        return False
    _STATE["installed"] = True
    return True


def available() -> bool:
    """True once the tool is configured (the HIP runtime has started with it)."""
    return _STATE["installed"] and _load().pa_tracer_available() == 1


def error():
    return _STATE["error"]


def enable():
    if not available():
        raise RuntimeError(f"device tracer not available: {_STATE['error'] or 'install() before HIP init'}")
    if _load().pa_tracer_enable() != 0:
        raise RuntimeError("rocprofiler_start_context failed")


def disable():
    """Stop recording and flush the buffered records (synchronise the device first)."""
    if available():
        _load().pa_tracer_disable()


def flush():
    """Drain the buffered records of kernels that have completed so far (recording
    continues)."""
    if available():
        _load().pa_tracer_flush()


def now_ns() -> int:
    return int(_load().pa_tracer_now_ns())


def push_range(rid: int):
    if available():
        _load().pa_tracer_push_range(rid)


def pop_range():
    if available():
        _load().pa_tracer_pop_range()


def clear():
    if _LIB is not None:
        _LIB.pa_tracer_clear()


def dropped() -> int:
    return int(_load().pa_tracer_dropped()) if _LIB is not None else 0


_DEMANGLED: dict[str, str] = {}


def demangle(names):
    """Itanium-demangled kernel names (llvm-cxxfilt / c++filt when present)."""
    todo = [n for n in set(names) if n not in _DEMANGLED]
    tool = shutil.which("llvm-cxxfilt") or ("/opt/rocm/lib/llvm/bin/llvm-cxxfilt"
                                             if os.path.exists("/opt/rocm/lib/llvm/bin/llvm-cxxfilt") else None) \
        or shutil.which("c++filt")
    if todo and tool:
        try:
            r = subprocess.run([tool], input="\n".join(todo), capture_output=True, text=True, timeout=30)
            out = r.stdout.splitlines()
            if len(out) == len(todo):
                _DEMANGLED.update(zip(todo, out))
        except (OSError, subprocess.SubprocessError):
            pass
    return [_DEMANGLED.get(n, n) for n in names]


def records(demangled=True):
    """Kernel records collected so far: dicts with name, device, queue, start_ns,
    end_ns, dur_ns, correlation, range (the external correlation id; 0 = none),
    grid, block, lds, scratch."""
    if _LIB is None:
        return []
    lib = _LIB
    n = lib.pa_tracer_count()
    u = (ctypes.c_uint64 * 8)()
    i = (ctypes.c_int32 * 7)()
    buf = ctypes.create_string_buffer(1024)
    out = []
    for k in range(n):
        ln = lib.pa_tracer_get(k, u, i, buf, 1024)
        if ln < 0:
            break
        name = buf.value.decode(errors="replace")
        if ln >= 1024:  # long template names: fetch in full
            big = ctypes.create_string_buffer(ln + 1)
            lib.pa_tracer_get(k, u, i, big, ln + 1)
            name = big.value.decode(errors="replace")
        out.append({"name": name, "kernel_id": int(u[0]), "start_ns": int(u[1]), "end_ns": int(u[2]),
                    "dur_ns": int(u[2]) - int(u[1]), "correlation": int(u[3]), "range": int(u[4]),
                    "queue": int(u[5]), "lds": int(u[6]), "scratch": int(u[7]), "device": int(i[0]),
                    "grid": (int(i[1]), int(i[2]), int(i[3])), "block": (int(i[4]), int(i[5]), int(i[6]))})
    if demangled and out:
        for r, d in zip(out, demangle([r["name"] for r in out])):
            r["name"] = d
    return out


def summary(recs=None):
    """{kernel name: (calls, total_ms)} sorted by total time."""
    recs = records() if recs is None else recs
    agg: dict[str, list] = {}
    for r in recs:
        a = agg.setdefault(r["name"], [0, 0.0])
        a[0] += 1
        a[1] += r["dur_ns"] / 1e6
    return dict(sorted(((k, (c, t)) for k, (c, t) in agg.items()), key=lambda kv: -kv[1][1]))
