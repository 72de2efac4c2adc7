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
        self._watched = {}  # tag -> None (an input whose gradient the caller wants)
        self._input_grads = {}  # tag -> gradient of a watched input after backward

    # ------------------------------------------------------------------ record
    def _tag(self, t):
        tag = self._next
        self._next += 1
        t._pa_tape = (id(self), tag)
        return tag

    def watch(self, t):
        """Make ``t`` (a tensor produced outside this tape: a pipeline stage's received
        activation, a recompute segment's input) a differentiable input of the tape;
        after :meth:`backward` its gradient is :meth:`grad` (t)."""
        if not isinstance(t, torch.Tensor) or not t.is_floating_point():
            return t
        tag = self._tag(t)
        self._watched[tag] = None
        return t

    def grad(self, t):
        """Gradient of a watched input (None if nothing on the tape used it)."""
        tg = getattr(t, "_pa_tape", None)
        if tg is None or tg[0] != id(self):
            return None
        return self._input_grads.get(tg[1])

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

    def backward_multi(self, outputs, grads):
        """Reverse pass seeded with several outputs (a pipeline stage's activations with
        the gradients the next stage returned); ``None`` gradients seed ones."""
        from ..utils import strict as _strict

        seeds = {}
        for o, g in zip(outputs, grads):
            tg = getattr(o, "_pa_tape", None)
            if tg is None or tg[0] != id(self):
                continue  # not produced on this tape (e.g. an integer passthrough)
            g = _ones_like(o) if g is None else g
            seeds[tg[1]] = g if tg[1] not in seeds else _add(seeds[tg[1]], g)
        if _strict.counting():
            with _strict.region("tape:backward", native=False):
                return self._run(seeds)
        return self._run(seeds)

    def _backward(self, loss, grad=None):
        tg = getattr(loss, "_pa_tape", None)
        if tg is None or tg[0] != id(self):
            raise RuntimeError("tape.backward: the loss was not produced on this tape")
        return self._run({tg[1]: _ones_like(loss) if grad is None else grad})

    def _run(self, grads):
        run_before_backward()  # e.g. an optimizer update still running on a side stream
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
        # what is left are the gradients of tensors no entry produced: watched inputs
        self._input_grads = {t: g for t, g in grads.items() if t in self._watched}

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


def _ones_like(t):
    """The reverse pass's seed on the native fill kernel."""
    if t.is_cuda:
        from ..ops import oplib

        return oplib.full_like(t, 1.0)
    return torch.ones_like(t)


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


class _RecomputeFn:
    """One recorded entry for a whole segment ``fn(*args)`` whose activations are not
    kept: the forward runs the segment with recording suspended (its fused ops save
    nothing that outlives the call), the backward runs it AGAIN on a private tape --
    inputs watched -- and differentiates that tape with the segment outputs'
    gradients.  Parameters used inside get their gradients (main_grad / .grad) and
    grad-ready hooks from the inner tape.  The framework's activation recomputation
    (reference: python/paddle/fluid/backward.py builds the program's own backward;
    this is the tape analogue of torch.utils.checkpoint)."""

    @staticmethod
    def forward(ctx, fn, *args):
        ctx.fn = fn
        ctx.args = args
        # the re-run must draw the same random numbers (dropout masks)
        ctx.rng = torch.get_rng_state()
        ctx.cuda_rng = torch.cuda.get_rng_state() if torch.cuda.is_available() and torch.cuda.is_initialized() else None
        with suspended():
            out = fn(*args)
        ctx.single = not isinstance(out, tuple)
        return out

    @staticmethod
    def backward(ctx, *gs):
        inner = Tape()
        prev = current()
        _TLS.tape = inner
        rng = torch.get_rng_state()
        cuda_rng = torch.cuda.get_rng_state() if ctx.cuda_rng is not None else None
        torch.set_rng_state(ctx.rng)
        if ctx.cuda_rng is not None:
            torch.cuda.set_rng_state(ctx.cuda_rng)
        try:
            with torch.no_grad():
                # only the inputs the outer tape differentiates (activations) are watched;
                # constants (rotary tables, masks) stay plain tensors
                need = ctx.needs_input_grad[1:]
                args = [inner.watch(a.detach()) if n and isinstance(a, torch.Tensor) and a.is_floating_point() else a
                        for a, n in zip(ctx.args, need)]
                out = ctx.fn(*args)
        finally:
            _TLS.tape = prev
            torch.set_rng_state(rng)
            if cuda_rng is not None:
                torch.cuda.set_rng_state(cuda_rng)
        outs = (out,) if ctx.single else tuple(out)
        pairs = [(o, g) for o, g in zip(outs, gs) if g is not None and isinstance(o, torch.Tensor)]
        inner.backward_multi([o for o, _ in pairs], [g for _, g in pairs])
        res = [inner.grad(a) if n and isinstance(a, torch.Tensor) and a.is_floating_point() else None
               for a, n in zip(args, need)]
        ctx.args = None
        return (None, *res)


def checkpoint(fn, *args):
    """Activation recomputation on the framework tape: while recording, ``fn(*args)``
    becomes one entry that recomputes its forward inside the reverse pass; outside a
    recording (eager / inference) it is just ``fn(*args)``."""
    t = current()
    if t is None:
        return fn(*args)
    return t.apply(_RecomputeFn, fn, *args)


@contextlib.contextmanager
def suspended():
    """Run ops without recording them (and without keeping what they save)."""
    prev = current()
    _TLS.tape = None
    _TLS.suspended = getattr(_TLS, "suspended", 0) + 1
    try:
        with torch.no_grad():
            yield
    finally:
        _TLS.suspended -= 1
        _TLS.tape = prev


def is_suspended():
    return getattr(_TLS, "suspended", 0) > 0


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
    if is_suspended():
        # inside a recompute segment's forward: compute, keep nothing for a backward
        with torch.no_grad():
            return fn.forward(_Ctx(tuple(False for _ in args)), *args)
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
