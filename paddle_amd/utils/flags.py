"""gflags-compatible runtime flags, settable through ``FLAGS_<name>`` env vars.

Parity: the reference's gflags passed from Python via
``core.init_gflags(["--tryfromenv=..."])`` (python/paddle/fluid/__init__.py:121-137).
Names keep the reference meaning; MI355X-specific flags are added at the end.
"""
from __future__ import annotations

import os

_DEFAULTS = {
    "fraction_of_gpu_memory_to_use": 0.92,
    "fraction_of_cpu_memory_to_use": 1.0,
    "initial_cpu_memory_in_mb": 500,
    "use_pinned_memory": True,
    "init_allocated_mem": False,
    "free_idle_memory": False,
    "benchmark": False,
    "stash_forward": True,  # keep forward autograd graphs for auto-VJP grad ops (no forward re-run)
    "eager_delete_scope": True,
    "check_nan_inf": False,
    "use_mkldnn": False,
    "cpu_deterministic": False,
    "cudnn_deterministic": False,
    "paddle_num_threads": 1,
    "io_threadpool_size": 100,
    "dist_threadpool_size": 0,
    "rpc_deadline": 180000,
    "rpc_server_profile_period": 0,
    "rpc_server_profile_path": "./profile_ps",
    "workspace_size_MB": 4096,
    # MI355X additions
    "allocator_strategy": "buddy",  # the native C++ buddy allocator behind torch (paddle_amd/__init__.py); any other value keeps torch's caching allocator
    "use_hip_graph": False,
    "rccl_bucket_mb": 256,
    "executor_engine": "auto",  # fluid.Executor engine: "auto" (C++ executor for every program it can take), "python" (op interpreter) or "native"
    "strict_native": False,  # utils/strict.py: an ATen device kernel (or host fallback of the C++ executor) inside a framework region is an error
    "count_aten": False,  # utils/strict.py: count ATen device kernels per region without raising
    "strict_trace": False,  # utils/strict.py: record the framework call site of each counted ATen kernel
    "dp_comm": "rccl",  # data-parallel gradient path: "rccl" (framework communicators) or "direct" (parallel/direct.py peer kernels)
    "direct_max_bytes": 64 << 20,  # parallel/direct.py scratch staging per rank
    "direct_one_shot_bytes": 1 << 20,  # one-shot / two-shot all-reduce switch
    "direct_max_spins": 1 << 25,  # bounded signal-barrier spins before a peer is declared lost
    "defer_expert_wgrad": True,  # ops/grouped.py: experts' dW once per step over all micro-batches (ops/accum.py)
    "fp8_wgrad": False,  # ops/grouped.py: fp8 expert dW (measured slower, profiles/r5_moe_fp8_wgrad_NEGATIVE.md)
}

_values = {}


def _parse(v, default):
    if isinstance(default, bool):
        return str(v).lower() in ("1", "true", "yes", "on")
    if isinstance(default, int):
        return int(v)
    if isinstance(default, float):
        return float(v)
    return v


def _load_env():
    for k, d in _DEFAULTS.items():
        e = os.environ.get("FLAGS_" + k)
        _values[k] = _parse(e, d) if e is not None else d


_load_env()


def get(name):
    return _values.get(name, _DEFAULTS.get(name))


def set(name, value):  # noqa: A001
    _values[name] = _parse(value, _DEFAULTS.get(name, value)) if isinstance(value, str) else value


def set_flags(d):
    for k, v in d.items():
        set(k[6:] if k.startswith("FLAGS_") else k, v)


def get_flags(names):
    if isinstance(names, str):
        names = [names]
    return {("FLAGS_" + n if not n.startswith("FLAGS_") else n): get(n[6:] if n.startswith("FLAGS_") else n)
            for n in names}


def init_gflags(argv):
    """Accepts ``--tryfromenv=a,b`` and ``--name=value`` like the reference binding."""
    for a in argv:
        a = a.lstrip("-")
        if a.startswith("tryfromenv="):
            for n in a.split("=", 1)[1].split(","):
                e = os.environ.get("FLAGS_" + n)
                if e is not None:
                    set(n, e)
        elif "=" in a:
            k, v = a.split("=", 1)
            set(k, v)
    return True


def all_flags():
    return dict(_values)
