"""fluid.profiler (python/paddle/fluid/profiler.py:39-272)."""
from __future__ import annotations

import contextlib

from ..utils import profiler as _p

__all__ = ["cuda_profiler", "reset_profiler", "profiler", "start_profiler", "stop_profiler"]


@contextlib.contextmanager
def cuda_profiler(output_file=None, output_mode=None, config=None):
    """Kept for API parity; on MI355X run the process under ``rocprofv3`` instead."""
    yield


def reset_profiler():
    _p.reset()


def start_profiler(state):
    if state not in ("CPU", "GPU", "All"):
        raise ValueError("The state must be 'CPU' or 'GPU' or 'All'.")
    _p.start(state)


def stop_profiler(sorted_key=None, profile_path="/tmp/profile"):
    if sorted_key not in (None, "default", "calls", "total", "max", "min", "ave"):
        raise ValueError("The sorted_key must be None or in 'calls', 'total', 'max', 'min' and 'ave'")
    return _p.stop(sorted_key, profile_path)


@contextlib.contextmanager
def profiler(state, sorted_key=None, profile_path="/tmp/profile"):
    start_profiler(state)
    try:
        yield
    finally:
        stop_profiler(sorted_key, profile_path)
