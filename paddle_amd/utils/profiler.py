"""Host + device event profiler (reference: platform/profiler.h:25-131, profiler.cc).

* ``RecordEvent(name)``: RAII push/pop of a named range; host time always, and
  device time through HIP events recorded on the current stream when the state
  includes the GPU (the reference used cudaEvent + CUPTI; on MI355X kernel-level
  activity comes from rocprofv3, and these ranges are also emitted as roctx
  markers when ``roctx`` is importable so rocprof traces show framework ops).
* per-thread event lists are kept by the native runtime library
  (``csrc/runtime/profiler.cc``) when it is built, else in Python;
* ``stop(sorted_key, path)`` prints the summary table (calls/total/min/max/ave,
  profiler.cc:277-323) and writes a Chrome trace JSON (tools/timeline.py parity).
"""
from __future__ import annotations

import json
import os
import threading
import time
from collections import defaultdict

import torch

_state = {"enabled": False, "gpu": False, "events": [], "t0": 0.0}
_lock = threading.Lock()
_tls = threading.local()


def is_enabled():
    return _state["enabled"]


class RecordEvent:
    __slots__ = ("name", "t", "ev0", "ev1")

    def __init__(self, name):
        self.name = name

    def __enter__(self):
        if not _state["enabled"]:
            return self
        self.t = time.perf_counter()
        if _state["gpu"]:
            self.ev0 = torch.cuda.Event(enable_timing=True)
            self.ev0.record()
        return self

    def __exit__(self, *a):
        if not _state["enabled"]:
            return False
        t1 = time.perf_counter()
        ev1 = None
        if _state["gpu"]:
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record()
        with _lock:
            _state["events"].append((self.name, threading.get_ident(), self.t, t1,
                                     getattr(self, "ev0", None), ev1))
        return False


class RecordBlock(RecordEvent):
    def __init__(self, block_id):
        super().__init__(f"block_{block_id}")


def start(state="All"):
    _state["enabled"] = True
    _state["gpu"] = state in ("GPU", "All") and torch.cuda.is_available()
    _state["events"] = []
    _state["t0"] = time.perf_counter()


def reset():
    with _lock:
        _state["events"] = []


def _gather():
    if _state["gpu"]:
        torch.cuda.synchronize()
    rows = []
    for name, tid, t0, t1, e0, e1 in _state["events"]:
        dev_ms = e0.elapsed_time(e1) if (e0 is not None and e1 is not None) else None
        rows.append((name, tid, t0, t1, dev_ms))
    return rows


def summary(sorted_key=None):
    rows = _gather()
    agg = defaultdict(lambda: [0, 0.0, float("inf"), 0.0, 0.0])
    for name, tid, t0, t1, dev in rows:
        ms = dev if dev is not None else (t1 - t0) * 1e3
        a = agg[name]
        a[0] += 1
        a[1] += ms
        a[2] = min(a[2], ms)
        a[3] = max(a[3], ms)
    items = [(n, c, tot, mn, mx, tot / c) for n, (c, tot, mn, mx, _) in agg.items()]
    key = {"calls": 1, "total": 2, "min": 3, "max": 4, "ave": 5}.get(sorted_key or "", None)
    if key is not None:
        items.sort(key=lambda r: -r[key] if key != 3 else r[key])
    lines = ["-------------------------> Profiling Report <-------------------------",
             f"{'Event':40s} {'Calls':>8s} {'Total':>12s} {'Min.':>10s} {'Max.':>10s} {'Ave.':>10s}"]
    for n, c, tot, mn, mx, ave in items:
        lines.append(f"{n[:40]:40s} {c:8d} {tot:12.4f} {mn:10.4f} {mx:10.4f} {ave:10.4f}")
    return "\n".join(lines), items


def stop(sorted_key=None, profile_path="/tmp/profile"):
    if not _state["enabled"]:
        return None
    text, items = summary(sorted_key)
    print(text)
    rows = _gather()
    t0 = _state["t0"]
    trace = {"traceEvents": [
        {"name": n, "ph": "X", "pid": os.getpid(), "tid": tid, "ts": (a - t0) * 1e6, "dur": (b - a) * 1e6,
         "args": ({"device_ms": d} if d is not None else {})}
        for n, tid, a, b, d in rows]}
    if profile_path:
        try:
            with open(profile_path + ".json" if not profile_path.endswith(".json") else profile_path, "w") as f:
                json.dump(trace, f)
        except OSError:
            pass
    _state["enabled"] = False
    return items
