"""fluid.Executor (python/paddle/fluid/executor.py:256-474).

``run`` clones the program once per (program, feed, fetch) signature with feed/fetch
ops inserted (cached; the reference re-creates ops every call unless
``use_program_cache``), feeds numpy/LoDTensor values onto the executor's place and
runs the block on the C++ executor (``fluid/native_engine.py``; ``engine="auto"``,
the default, for every program it can take) or on the Python op interpreter
(:class:`paddle_amd.framework.executor.BlockExecutor`: step-scope control flow,
SelectedRows / RPC programs, ``engine="python"``), then fetches results (the only
host sync).

``Executor(place, use_hip_graph=True)`` additionally captures a steady-state step
of a static-shape program into a HIP graph and replays it (MI355X-first
replacement for launch-bound inner loops; see also ``FLAGS_use_hip_graph``).

The default engine is ``"auto"`` (``FLAGS_executor_engine``): the C++ executor of
``csrc/native`` (:mod:`paddle_amd.fluid.native_engine`, reference
framework/executor.cc:125-353) for every program it can take.
``Executor(place, engine="native")`` forces the C++ executor;
programs it cannot take (sub-blocks needing step scopes, non-LoDTensor variables)
raise.  ``engine="auto"`` runs every program the C++ executor can take on it (ops
without a C++ kernel run their Python kernel per op) and the rest -- and runs
that need the interpreter's per-op hooks (profiler, NaN/Inf checks, VLOG op
traces, HIP-graph capture, py_reader feeds) -- on the interpreter.
"""
from __future__ import annotations

import contextlib

import numpy as np
import torch

from ..framework import core
from ..framework.executor import BlockExecutor
from ..utils import flags as FLAGS
from .framework import Program, Variable, default_main_program

g_scope = core.global_scope()


def global_scope():
    return core.global_scope()


@contextlib.contextmanager
def scope_guard(scope):
    old = core._switch_scope(scope)
    try:
        yield
    finally:
        core._switch_scope(old)


def _to_lod_tensor(data, place):
    if isinstance(data, core.LoDTensor):
        return data
    if isinstance(data, torch.Tensor):
        return core.LoDTensor(data.to(place.torch_device()))
    arr = np.asarray(data)
    t = torch.from_numpy(np.ascontiguousarray(arr))
    if place.torch_device().type == "cuda":
        t = t.pin_memory().to(place.torch_device(), non_blocking=True)
    return core.LoDTensor(t)


def as_numpy(tensor):
    if isinstance(tensor, list):
        return [as_numpy(t) for t in tensor]
    if isinstance(tensor, core.LoDTensor):
        if tensor.lod() and False:
            raise RuntimeError("Some of your fetched tensors hold LoD information")
        return tensor.numpy()
    if isinstance(tensor, core.SelectedRows):
        return tensor.get_tensor().numpy()
    return np.asarray(tensor)


class Executor:
    def __init__(self, place=None, use_hip_graph=None, engine=None):
        self.place = place or core.CPUPlace()
        self._core = BlockExecutor(self.place)
        self.engine = engine or FLAGS.get("executor_engine") or "python"
        if self.engine not in ("python", "native", "auto"):
            raise ValueError(f"unknown executor engine {self.engine!r}")
        self._native = None
        self._auto = {}  # (id(program), version) -> (program, takes native)
        self._closed = False
        self._prog_cache = {}
        self.use_hip_graph = FLAGS.get("use_hip_graph") if use_hip_graph is None else use_hip_graph

    def close(self):
        """Reference executor.py close(): tell every parameter server this trainer
        talked to that it is done (SendComplete), so sync pservers can exit."""
        import sys

        if not self._closed and "paddle_amd.distributed.ps.rpc" in sys.modules:
            from ..distributed.ps import RPCClient

            c = RPCClient.instance()
            if c.endpoints:
                c.complete(sorted(c.endpoints))
                c.endpoints.clear()
        self._closed = True

    def as_lodtensor(self, data):
        return _to_lod_tensor(data, self.place)

    def _add_feed_fetch_ops(self, program, feed, fetch_list, feed_var_name, fetch_var_name):
        tmp = program.clone()
        gb = tmp.global_block()
        if feed_var_name in gb.vars:
            feed_var = gb.vars[feed_var_name]
        else:
            feed_var = gb.create_var(name=feed_var_name, type=core.VT.FEED_MINIBATCH, persistable=True)
        if fetch_var_name in gb.vars:
            fetch_var = gb.vars[fetch_var_name]
        else:
            fetch_var = gb.create_var(name=fetch_var_name, type=core.VT.FETCH_LIST, persistable=True)
        if not any(op.type == "feed" for op in gb.ops):
            for i, name in enumerate(feed):
                out = gb.var(name)
                gb.prepend_op(type="feed", inputs={"X": [feed_var]}, outputs={"Out": [out]}, attrs={"col": i})
        if not any(op.type == "fetch" for op in gb.ops):
            for i, var in enumerate(fetch_list):
                gb.append_op(type="fetch", inputs={"X": [var]}, outputs={"Out": [fetch_var]}, attrs={"col": i})
        return tmp

    def run(self, program=None, feed=None, fetch_list=None, feed_var_name="feed", fetch_var_name="fetch",
            scope=None, return_numpy=True, use_program_cache=False):
        if self._closed:
            raise RuntimeError("Attempted to use a closed Executor")
        if feed is None:
            feed = {}
        if fetch_list is None:
            fetch_list = []
        if program is None:
            program = default_main_program()
        if hasattr(program, "_compiled_program"):
            program = program._compiled_program
        if not isinstance(program, Program):
            raise TypeError("Executor requires Program as its Parameter")
        if scope is None:
            scope = global_scope()
        readers = getattr(program, "_py_readers", None)
        if readers:
            # py_reader programs run without a feed: each started reader supplies the
            # next batch of its data vars (EOFException once it is exhausted)
            feed = dict(feed)
            for r in readers:
                if r.started and not all(v.name in feed for v in r.feed_vars):
                    feed.update(r.next_feed())
        fetch_names = [v.name if isinstance(v, Variable) else str(v) for v in fetch_list]
        feed_names = list(feed.keys())
        if self.engine != "python" and program.global_block().ops and (
                self.engine == "native" or self._auto_native(program, feed, readers)):
            if self._native is None:
                from .native_engine import NativeEngine

                self._native = NativeEngine(self.place)
            return self._native.run(program, feed, fetch_names, scope, return_numpy)
        key = (id(program), program._version, tuple(feed_names), tuple(fetch_names), feed_var_name, fetch_var_name)
        prog = self._prog_cache.get(key)
        if prog is None:
            prog = self._add_feed_fetch_ops(program, feed_names, fetch_names, feed_var_name, fetch_var_name)
            self._prog_cache[key] = prog
        # feed
        feed_list = [None] * len(feed_names)
        gb = prog.global_block()
        for op in gb.ops:
            if op.type == "feed":
                name = op.output("Out")[0]
                feed_list[op.attrs["col"]] = _to_lod_tensor(feed[name], self.place)
        scope.var(feed_var_name).set(feed_list)
        scope.var(fetch_var_name).set([])
        self._core.run_block(prog, 0, scope)
        outs = scope.find_var(fetch_var_name).get() or []
        if return_numpy:
            return [as_numpy(o) for o in outs]
        return outs

    def _auto_native(self, program, feed, readers):
        """engine="auto": does this run go to the C++ executor?"""
        from .. import platform as _platform
        from ..utils import profiler as _prof

        if (readers or self.use_hip_graph or FLAGS.get("check_nan_inf") or _prof.is_enabled()
                or _platform.vlog_level() >= 1):
            return False
        key = (id(program), program._version)
        ent = self._auto.get(key)
        if ent is None or ent[0] is not program:
            from .native_engine import NativeEngine

            ent = (program, NativeEngine.can_run(program, self.place))
            self._auto[key] = ent
        if not ent[1]:
            return False
        for v in feed.values():
            t = v._t if isinstance(v, core.LoDTensor) else v
            dt = getattr(t, "dtype", None)
            if dt is not None and str(dt).replace("torch.", "") not in (
                    "float32", "float64", "int32", "int64", "float16", "bfloat16", "uint8", "int8", "bool"):
                return False
        return True

    def _run_block(self, program, block_idx, scope):
        self._core.run_block(program, block_idx, scope)
