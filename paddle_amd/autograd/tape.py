"""The framework's own reverse-mode tape for the fused-op path (torch autograd off).

Reference: the DyGraph tracer + autograd engine (paddle/fluid/imperative/tracer.cc,
engine.cc in later Paddle; the 0.14 snapshot differentiates Programs with
backward.py).  Every op on the LLaMA / GPT / MoE path is a fused kernel with a
hand-written backward (``ops.fused`` Functions).  Under ``recording()``:

  * forward runs with torch's grad mode OFF: each fused op calls its Function's
    ``forward`` directly with a light context object, and the tape records
    (Function, context, input handles, output ids);
  * ``Tape.backward(loss)`` walks the records in reverse, calls each
    ``backward`` with the gradients of its outputs, accumulates input gradients by
    tape id (activations) or into ``param.grad`` (parameters whose fused backward
    did not already write the sharded optimizer's fp32 ``main_grad``);
  * a parameter's grad-ready hooks (``param._pa_grad_ready_hooks``: the sharded
    optimizer's bucket accounting / reduce-scatter launch) fire when its LAST use
    on the tape has been differentiated -- the post-accumulate-grad contract.

Activations are tracked by an integer tag stored on the tensor, not by strong
references, so the tape keeps alive only what the Functions themselves save.
"""
from __future__ import annotations

import contextlib
import threading
import weakref

import torch

_TLS = threading.local()


def current():
    return getattr(_TLS, "tape", None)


class _Ctx:
    """Stands in for torch's FunctionCtx inside Function.forward / backward."""

    __slots__ = ("needs_input_grad", "saved_tensors", "__dict__")

    def __init__(self, needs):
        self.needs_input_grad = needs
        self.saved_tensors = ()

    def save_for_backward(self, *ts):
        self.saved_tensors = ts

    def mark_non_differentiable(self, *ts):
        pass

    def set_materialize_grads(self, v):
        pass

    def mark_dirty(self, *ts):
        pass


class _Entry:
    __slots__ = ("fn", "ctx", "inputs", "outputs")

    def __init__(self, fn, ctx, inputs, outputs):
        self.fn, self.ctx, self.inputs, self.outputs = fn, ctx, inputs, outputs


class Tape:
    def __init__(self):
        self.entries: list[_Entry] = []
        self._next = 1
        self._uses = {}     # id(param) -> remaining uses on the tape
        self._params = {}   # id(param) -> param

    # ------------------------------------------------------------------ record
    def _tag(self, t):
        tag = self._next
        self._next += 1
        t._pa_tape = (id(self), tag)
        return tag

    def _handle(self, a):
        """('act', tag) for a tracked activation, ('param', p) for a leaf that
        requires grad, None otherwise."""
        if not isinstance(a, torch.Tensor):
            return None
        tg = getattr(a, "_pa_tape", None)
        if tg is not None and tg[0] == id(self):
            return ("act", tg[1])
        if a.requires_grad and a.is_leaf:
            self._uses[id(a)] = self._uses.get(id(a), 0) + 1
            self._params[id(a)] = a
            return ("param", a)
        return None

    def apply(self, fn, *args):
        handles = [self._handle(a) for a in args]
        for a, h in zip(args, handles):
            # a parameter reached this op through an op the tape did not record (a
            # view such as w.t(), or any plain torch op): its gradient would be lost
            if h is None and isinstance(a, torch.Tensor) and a.is_floating_point():
                base = a._base
                if base is not None and (base.requires_grad or getattr(base, "_pa_tape", (None,))[0] == id(self)):
                    raise RuntimeError(
                        f"tape: an input of {getattr(fn, '__name__', fn)} is a view of a parameter or recorded "
                        "activation taken outside the tape; its gradient would be dropped. Use a fused op "
                        "(e.g. ops.linear_t for x @ W^T) instead of the plain torch view.")
        ctx = _Ctx(tuple(h is not None for h in handles))
        with torch.no_grad():
            outs = fn.forward(ctx, *args)
        single = not isinstance(outs, tuple)
        tup = (outs,) if single else outs
        out_tags = [self._tag(o) if isinstance(o, torch.Tensor) and o.is_floating_point() else None for o in tup]
        if any(h is not None for h in handles):
            self.entries.append(_Entry(fn, ctx, handles, out_tags))
        return outs

    # ------------------------------------------------------------------ backward
    def backward(self, loss, grad=None):
        from ..utils import strict as _strict

        if _strict.counting():
            # strict-native accounting of the reverse pass (the fused ops' backwards)
            with _strict.region("tape:backward", native=False):
                return self._backward(loss, grad)
        return self._backward(loss, grad)

    def _backward(self, loss, grad=None):
        run_before_backward()  # e.g. an optimizer update still running on a side stream
        tg = getattr(loss, "_pa_tape", None)
        if tg is None or tg[0] != id(self):
            raise RuntimeError("tape.backward: the loss was not produced on this tape")
        grads = {tg[1]: torch.ones_like(loss) if grad is None else grad}
        with torch.no_grad():
            for e in reversed(self.entries):
                outg = [grads.pop(t, None) if t is not None else None for t in e.outputs]
                if all(g is None for g in outg):
                    self._release(e)
                    continue
                res = e.fn.backward(e.ctx, *outg)
                if not isinstance(res, tuple):
                    res = (res,)
                for h, g in zip(e.inputs, res):
                    if h is None:
                        continue
                    if h[0] == "act":
                        if g is not None:
                            prev = grads.get(h[1])
                            grads[h[1]] = g if prev is None else _add(prev, g)
                    else:
                        p = h[1]
                        if g is not None:
                            g = g.to(p.dtype)
                            p.grad = g if p.grad is None else _add(p.grad, g)
                        self._param_done(p)
                e.ctx = None
        self.entries.clear()

    def _release(self, e):
        for h in e.inputs:
            if h is not None and h[0] == "param":
                self._param_done(h[1])
        e.ctx = None

    def _param_done(self, p):
        k = id(p)
        n = self._uses.get(k, 0) - 1
        self._uses[k] = n
        if n == 0:
            for hook in getattr(p, "_pa_grad_ready_hooks", ()):
                hook(p)


def _add(a, b):
    """Gradient accumulation on the op library's broadcast kernel (oplib.hip)."""
    if a.is_cuda and a.shape == b.shape and a.dtype == b.dtype:
        from ..ops import oplib

        r = oplib.binary("add", a, b)
        if r is not None:
            return r
    return a + b


# pending callbacks, held weakly: a bound method of an optimizer that is gone (or
# that already drained its own wait) must not keep it and its buffers alive
_BEFORE_BACKWARD = []


def before_next_backward(fn):
    """Run ``fn`` once at the start of the next reverse pass (before any gradient
    is written) -- of this tape, of the eager engine, or of torch autograd."""
    ref = weakref.WeakMethod(fn) if hasattr(fn, "__self__") else (lambda f=fn: f)
    for r in _BEFORE_BACKWARD:
        if r() == fn:
            return
    _BEFORE_BACKWARD.append(ref)


def run_before_backward():
    """Drain the pending callbacks (every reverse-pass entry point calls this)."""
    while _BEFORE_BACKWARD:
        fn = _BEFORE_BACKWARD.pop(0)()
        if fn is not None:
            fn()


def cancel_before_backward(fn):
    """Drop a pending callback (its owner already waited for what it guards)."""
    _BEFORE_BACKWARD[:] = [r for r in _BEFORE_BACKWARD if r() is not None and r() != fn]


@contextlib.contextmanager
def recording():
    """Record fused ops on a fresh tape with torch autograd disabled; yields the tape."""
    prev = current()
    t = Tape()
    _TLS.tape = t
    try:
        with torch.no_grad():
            yield t
    finally:
        _TLS.tape = prev


def apply(fn, *args):
    """Application of a fused op ``fn`` (hand-written forward / backward):

    * on the active tape (bench / model step recording), if any;
    * else, when an argument is a framework ``Tensor`` (DyGraph), on the eager
      engine: one grad node whose backward is ``fn.backward`` (torch autograd off);
    * else (raw torch tensors: interop with torch-native code) ``fn.apply``."""
    t = current()
    if t is not None:
        return t.apply(fn, *args)
    from . import engine

    if any(isinstance(a, engine.Tensor) for a in args):
        if engine.is_grad_enabled():
            out = engine.record_function(fn, args)
            if out is not None:
                return out
        ctx = _Ctx(tuple(False for _ in args))
        with torch.no_grad(), torch._C.DisableTorchFunctionSubclass():
            out = fn.forward(ctx, *[engine._raw(a) for a in args])
        return engine._wrap(out)
    return fn.apply(*args)
