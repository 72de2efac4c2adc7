"""SSA-graph multi-device execution (reference: paddle/fluid/framework/details/ --
multi_devices_graph_pass.cc:320-700 builds one graph of per-device
ComputationOpHandles plus AllReduce / Reduce / Broadcast handles,
threaded_ssa_graph_executor.cc:36-211 runs it on a thread pool as dependencies
resolve, all_reduce_op_handle.cc:99 syncs one gradient).

MI355X-first differences:
  * gradients are synchronised in BUCKETS (FLAGS_rccl_bucket_mb, filled in
    backward-production order): one flat all-reduce per bucket over RCCL, issued
    the moment the last producer of the bucket's last gradient has run on every
    replica -- so the all-reduce of late layers overlaps the backward of early
    ones (the reference issues one ncclAllReduce per gradient);
  * communication runs on its own HIP stream per device, ordered against the
    compute stream with events (record after the producers, wait before the
    consumers) instead of device-wide syncs;
  * the graph runs on the native C++ DAG scheduler (csrc/runtime/threading.cc,
    ``runtime.dag_run``) with one worker per replica plus one for communication.
"""
from __future__ import annotations

import threading
import time
from collections import defaultdict

import torch


def op_deps(ops):
    """deps[j] = indices of earlier ops that op j must follow: read-after-write,
    write-after-read and write-after-write on variable names (program order)."""
    last_w = {}
    readers = defaultdict(list)
    deps = []
    for j, op in enumerate(ops):
        d = set()
        for n in op.input_arg_names:
            if n in last_w:
                d.add(last_w[n])
        for n in op.output_arg_names:
            if n in last_w:
                d.add(last_w[n])
            d.update(readers.get(n, ()))
        d.discard(j)
        deps.append(d)
        for n in op.input_arg_names:
            readers[n].append(j)
        for n in op.output_arg_names:
            last_w[n] = j
            readers[n] = []
    return deps


class Node:
    __slots__ = ("kind", "replica", "index", "fn", "name")

    def __init__(self, kind, replica, index, fn, name):
        self.kind, self.replica, self.index, self.fn, self.name = kind, replica, index, fn, name


class SSAGraph:
    """Nodes + edges (u before v) of one training step."""

    def __init__(self):
        self.nodes: list[Node] = []
        self.edges: list[tuple[int, int]] = []

    def add(self, kind, replica, index, fn, name):
        self.nodes.append(Node(kind, replica, index, fn, name))
        return len(self.nodes) - 1

    def edge(self, u, v):
        if u != v:
            self.edges.append((u, v))


class Trace:
    """Per-node (start, end, thread) records of the last step (for timelines / tests)."""

    def __init__(self):
        self.events = []
        self._lock = threading.Lock()

    def add(self, node, t0, t1):
        with self._lock:
            self.events.append((node.kind, node.name, node.replica, t0, t1, threading.get_ident()))


def run_graph(graph: SSAGraph, nthreads: int, trace: Trace | None = None):
    from .. import runtime

    def fn(i):
        node = graph.nodes[i]
        t0 = time.perf_counter()
        node.fn()
        if trace is not None:
            trace.add(node, t0, time.perf_counter())

    if runtime.available():
        runtime.dag_run(len(graph.nodes), graph.edges, fn, nthreads=nthreads)
        return
    # host fallback: Kahn order on the calling thread
    indeg = [0] * len(graph.nodes)
    succ = defaultdict(list)
    for u, v in graph.edges:
        succ[u].append(v)
        indeg[v] += 1
    ready = [i for i, d in enumerate(indeg) if d == 0]
    while ready:
        i = ready.pop(0)
        fn(i)
        for v in succ[i]:
            indeg[v] -= 1
            if indeg[v] == 0:
                ready.append(v)


class StreamSet:
    """Compute stream (torch's current) and a communication stream per CUDA device."""

    def __init__(self):
        self._comm = {}

    def comm(self, dev):
        s = self._comm.get(dev)
        if s is None:
            from ..platform import device_context

            dc = device_context(dev)  # the device context's high-priority comm stream
            s = self._comm[dev] = dc.comm_stream if dc is not None else torch.cuda.Stream(device=dev)
        return s
