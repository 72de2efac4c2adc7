"""Host + device event profiler (reference: platform/profiler.h:25-131, profiler.cc).

* ``RecordEvent(name)``: RAII push/pop of a named range; host time always, and
  device time through HIP events recorded on the current stream when the state
  includes the GPU (the reference used cudaEvent + CUPTI; on MI355X kernel-level
  activity comes from rocprofv3, and these ranges are also emitted as roctx
  markers when ``roctx`` is importable so rocprof traces show framework ops).
* with the rocprofiler-sdk kernel tracer installed (``utils/device_tracer.py``,
  ``FLAGS_device_tracer=1``; the reference's CUPTI DeviceTracer), every kernel the
  process dispatches inside the profiling window is recorded in-process with its
  device start/end time and the innermost enclosing RecordEvent, and the GPU
  track of the profile is those kernels;
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

_state = {"enabled": False, "gpu": False, "events": [], "t0": 0.0, "base": None, "tracer": False,
          "ranges": {}, "next_range": 1}
_lock = threading.Lock()
_tls = threading.local()


def is_enabled():
    return _state["enabled"]


def _tracer():
    from . import device_tracer

    return device_tracer


class RecordEvent:
    __slots__ = ("name", "t", "ev0", "ev1", "rid")

    def __init__(self, name):
        self.name = name
        self.rid = 0

    def __enter__(self):
        if not _state["enabled"]:
            return self
        if _state["tracer"]:
            with _lock:
                self.rid = _state["next_range"]
                _state["next_range"] += 1
                _state["ranges"][self.rid] = self.name
            _tracer().push_range(self.rid)
        self.t = time.perf_counter()
        if _state["gpu"]:
            self.ev0 = torch.cuda.Event(enable_timing=True)
            self.ev0.record()
        return self

    def __exit__(self, *a):
        if not _state["enabled"]:
            return False
        t1 = time.perf_counter()
        if self.rid:
            _tracer().pop_range()
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
    _state["tracer"] = False
    if state in ("GPU", "All"):
        try:
            dt = _tracer()
            if dt.available():
                dt.clear()
                _state["ranges"], _state["next_range"] = {}, 1
                _state["tracer_t0"] = (time.perf_counter(), dt.now_ns())
                dt.enable()
                _state["tracer"] = True
        except (OSError, RuntimeError):
            _state["tracer"] = False
    if _state["gpu"]:
        # device time origin: every range's HIP events are placed relative to it, so
        # the GPU track of the timeline is an in-process device activity trace
        # (the reference's CUPTI DeviceTracer, platform/device_tracer.cc:98-121)
        _state["base"] = torch.cuda.Event(enable_timing=True)
        _state["base"].record()
        torch.cuda.synchronize()
        _state["base_host"] = time.perf_counter()


def reset():
    with _lock:
        _state["events"] = []


def kernel_records():
    """The in-process kernel records of the window (empty without the tracer).
    Inside an open window the device is synchronised and the buffer flushed first."""
    if _state.get("tracer"):
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        _tracer().flush()
    elif not _state.get("tracer_used"):
        return []
    recs = _tracer().records()
    for r in recs:
        r["op"] = _state["ranges"].get(r["range"], "")
    return recs


def _stop_tracer():
    if _state["tracer"]:
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        _tracer().disable()
        _state["tracer"] = False
        _state["tracer_used"] = True


def _gather():
    if _state["gpu"]:
        torch.cuda.synchronize()
    rows = []
    for name, tid, t0, t1, e0, e1 in _state["events"]:
        dev_ms = e0.elapsed_time(e1) if (e0 is not None and e1 is not None) else None
        rows.append((name, tid, t0, t1, dev_ms))
    return rows


def device_events():
    """(name, device_start_ms, device_end_ms) of every GPU range, on the device clock
    measured from the profiler start event."""
    if not _state["gpu"] or _state["base"] is None:
        return []
    torch.cuda.synchronize()
    base = _state["base"]
    out = []
    for name, tid, t0, t1, e0, e1 in _state["events"]:
        if e0 is not None and e1 is not None:
            out.append((name, base.elapsed_time(e0), base.elapsed_time(e1)))
    return out


def profile_dict():
    """The profile as a plain dict (the reference's profiler.proto Profile):
    ``events``: {name, type CPU|GPUKernel, device_id, sub_device_id (thread /
    stream), start_ns, end_ns}."""
    t0 = _state["t0"]
    ev = [{"name": n, "type": "CPU", "device_id": 0, "sub_device_id": tid % 1000000,
           "start_ns": int((a - t0) * 1e9), "end_ns": int((b - t0) * 1e9)} for n, tid, a, b, _ in _gather()]
    _stop_tracer()
    krecs = kernel_records()
    if krecs:
        # kernels on the host clock: rocprofiler ns mapped through the (perf_counter,
        # rocprofiler ns) pair taken at start(); one sub-track per HIP queue
        h0, d0 = _state["tracer_t0"]
        qs = {q: i for i, q in enumerate(sorted({r["queue"] for r in krecs}))}
        ev += [{"name": r["name"], "type": "GPUKernel", "device_id": max(r["device"], 0),
                "sub_device_id": qs[r["queue"]], "op": r["op"],
                "start_ns": int((h0 - t0) * 1e9) + r["start_ns"] - d0,
                "end_ns": int((h0 - t0) * 1e9) + r["end_ns"] - d0} for r in krecs]
    elif _state["gpu"]:
        off = (_state["base_host"] - t0) * 1e3
        dev = torch.cuda.current_device()
        ev += [{"name": n, "type": "GPUKernel", "device_id": dev, "sub_device_id": 0,
                "start_ns": int((off + a) * 1e6), "end_ns": int((off + b) * 1e6)} for n, a, b in device_events()]
    return {"start_ns": 0, "end_ns": max([e["end_ns"] for e in ev], default=0), "events": ev}


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
    _stop_tracer()
    text, items = summary(sorted_key)
    print(text)
    if profile_path:
        # the profile itself (tools/timeline.py turns one or more into a Chrome
        # trace), plus the single-process Chrome trace next to it
        try:
            prof = profile_dict()
            with open(profile_path, "w") as f:
                json.dump(prof, f)
            with open(profile_path + ".trace.json", "w") as f:
                f.write(chrome_trace({"trainer": prof}))
        except OSError:
            pass
    _state["enabled"] = False
    return items


def chrome_trace(profiles):
    """Chrome trace JSON of {label: profile_dict} (tools/timeline.py Timeline):
    one pid per (label, device, CPU | GPUKernel) track, tid = sub_device_id."""
    pids, out = {}, []
    for k, prof in profiles.items():
        for e in prof["events"]:
            key = (k, e["device_id"], e["type"])
            if key not in pids:
                pids[key] = len(pids)
                kind = "cpu:block" if e["type"] == "CPU" else "gpu"
                out.append({"name": "process_name", "ph": "M", "pid": pids[key],
                            "args": {"name": f"{k}:{kind}:{e['device_id']}"}})
            out.append({"name": e["name"], "cat": "Op", "ph": "X", "pid": pids[key], "tid": e["sub_device_id"],
                        "ts": e["start_ns"] / 1e3, "dur": (e["end_ns"] - e["start_ns"]) / 1e3,
                        "args": {"name": e["name"], **({"op": e["op"]} if e.get("op") else {})}})
    return json.dumps({"traceEvents": out, "displayTimeUnit": "ns"})
