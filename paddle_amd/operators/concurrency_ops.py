"""CSP concurrency operators (reference: framework/channel.h, channel_impl.h and
operators/{channel_create,channel_send,channel_recv,channel_close,go,select}_op.cc).

* A channel is a host object holding LoDTensors: buffered (capacity > 0) sends
  block only when full; unbuffered (capacity 0) sends rendezvous with a receiver.
  ``close`` wakes every waiter: pending and later sends fail (Status False),
  receives drain what is buffered and then return Status False with a zero value.
* ``go`` runs its sub-block on a new host thread in a child scope (goroutine);
  device work it issues goes to that thread's current HIP stream.
* ``select`` blocks until one case's channel operation can proceed (or runs the
  default case), performs it, records the chosen case index and runs the
  sub-block whose per-case conditional blocks key on that index.
"""
from __future__ import annotations

import threading

import torch

from ..framework import core
from ..framework.registry import register_op


class Channel:
    def __init__(self, capacity=0, dtype=None):
        self.capacity = int(capacity)
        self.dtype = dtype
        self._buf = []
        self._closed = False
        self._cv = threading.Condition()
        self._recv_waiting = 0      # receivers parked (for unbuffered rendezvous)
        self._taken = 0             # unbuffered: items handed over so far
        self._put = 0

    # ---------------------------------------------------------------- state probes
    def can_send(self):
        with self._cv:
            if self._closed:
                return True          # a send on a closed channel "proceeds" (and fails)
            if self.capacity > 0:
                return len(self._buf) < self.capacity
            return self._recv_waiting > len(self._buf)

    def can_recv(self):
        with self._cv:
            return bool(self._buf) or self._closed

    # ---------------------------------------------------------------- operations
    def send(self, value):
        with self._cv:
            if self._closed:
                return False
            if self.capacity > 0:
                while len(self._buf) >= self.capacity and not self._closed:
                    self._cv.wait()
                if self._closed:
                    return False
                self._buf.append(value)
                self._cv.notify_all()
                return True
            # unbuffered: enqueue, then wait until a receiver has taken it
            self._buf.append(value)
            self._put += 1
            ticket = self._put
            self._cv.notify_all()
            while self._taken < ticket and not self._closed:
                self._cv.wait()
            if self._taken < ticket:      # closed before hand-over: withdraw
                self._buf = [x for x in self._buf if x is not value]
                return False
            return True

    def recv(self):
        with self._cv:
            self._recv_waiting += 1
            self._cv.notify_all()
            try:
                while not self._buf and not self._closed:
                    self._cv.wait()
                if not self._buf:
                    return None, False
                v = self._buf.pop(0)
                self._taken += 1
                self._cv.notify_all()
                return v, True
            finally:
                self._recv_waiting -= 1

    def close(self):
        with self._cv:
            self._closed = True
            self._cv.notify_all()

    def wait_any(self, timeout=0.05):
        with self._cv:
            self._cv.wait(timeout)


def _chan(ctx, slot="Channel"):
    c = ctx.input_value(slot)
    if not isinstance(c, Channel):
        raise RuntimeError(f"{ctx.op.type}: input {slot} is not a channel (did channel_create run?)")
    return c


@register_op("channel_create", [], ["Out"], {"data_type": 5, "capacity": 0}, grad=None, no_infer=True,
             share_lod=False)
def channel_create(ctx):
    ctx.set_output("Out", Channel(ctx.attr("capacity"), ctx.attr("data_type")))


@register_op("channel_close", ["Channel"], [], {}, grad=None, no_infer=True, share_lod=False)
def channel_close(ctx):
    _chan(ctx).close()


def _snapshot(v):
    if isinstance(v, core.LoDTensor):
        return core.LoDTensor(v.tensor.clone(), v.lod())
    if isinstance(v, torch.Tensor):
        return core.LoDTensor(v.clone())
    return v


@register_op("channel_send", ["Channel", "X"], ["Status?"], {"is_copy": False}, grad=None, no_infer=True,
             share_lod=False)
def channel_send(ctx):
    ok = _chan(ctx).send(_snapshot(ctx.input_value("X")))
    if ctx.has_output("Status"):
        ctx.set_output("Status", torch.tensor([ok], dtype=torch.bool))


def _zero_like_dtype(ch):
    dt = core.to_torch_dtype(ch.dtype) if isinstance(ch.dtype, int) else torch.float32
    return core.LoDTensor(torch.zeros(1, dtype=dt))


@register_op("channel_recv", ["Channel"], ["Out", "Status?"], {}, grad=None, no_infer=True, share_lod=False)
def channel_recv(ctx):
    ch = _chan(ctx)
    v, ok = ch.recv()
    ctx.set_output("Out", v if ok else _zero_like_dtype(ch))
    if ctx.has_output("Status"):
        ctx.set_output("Status", torch.tensor([ok], dtype=torch.bool))


@register_op("go", ["X*?"], [], {"sub_block": None}, grad=None, no_infer=True, share_lod=False)
def go_op(ctx):
    """Launch the sub-block on a new thread in a child scope (go_op.cc ExecuteOnThread)."""
    blk, scope, exe = ctx.attr("sub_block"), ctx.scope, ctx.executor
    child = scope.new_scope()
    dev = torch.cuda.current_device() if torch.cuda.is_available() else None

    def run():
        if dev is not None:
            torch.cuda.set_device(dev)
        exe.run_block(blk.program, blk.idx, child)

    t = threading.Thread(target=run, daemon=True, name="paddle_amd_go")
    t.start()
    _GO_THREADS.append(t)


_GO_THREADS: list = []


def join_go_threads(timeout=None):
    """Wait for every goroutine launched so far (tests / clean shutdown)."""
    for t in list(_GO_THREADS):
        t.join(timeout)
    _GO_THREADS[:] = [t for t in _GO_THREADS if t.is_alive()]


@register_op("select", ["X*?", "case_to_execute"], ["Out*?"], {"sub_block": None, "cases": []}, grad=None,
             no_infer=True, share_lod=False)
def select_op(ctx):
    """cases: strings "idx,action,channel,value" with action 0=default 1=send 2=recv."""
    scope, exe = ctx.scope, ctx.executor
    cases = []
    for c in ctx.attr("cases"):
        idx, act, ch, val = c.split(",")
        cases.append((int(idx), int(act), ch, val))
    default = next((c for c in cases if c[1] == 0), None)
    chosen = None
    while chosen is None:
        for idx, act, chn, val in cases:
            if act == 0:
                continue
            ch = scope.find_var(chn).get()
            if (act == 1 and ch.can_send()) or (act == 2 and ch.can_recv()):
                chosen = (idx, act, ch, val)
                break
        if chosen is None:
            if default is not None:
                chosen = (default[0], 0, None, None)
                break
            # park briefly on any channel of the select, then re-poll
            first = next(c for c in cases if c[1] != 0)
            scope.find_var(first[2]).get().wait_any()
    idx, act, ch, val = chosen
    if act == 1:
        ch.send(_snapshot(scope.find_var(val).get()))
    elif act == 2:
        v, ok = ch.recv()
        scope.find_var(val).set(v if ok else _zero_like_dtype(ch))
    cv = scope.find_var(ctx.op.input("case_to_execute")[0])
    cv.set(core.LoDTensor(torch.tensor([idx], dtype=torch.int32)))
    blk = ctx.attr("sub_block")
    exe.run_block(blk.program, blk.idx, scope.new_scope())
