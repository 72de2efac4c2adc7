"""DyGraph eager autograd engine: the framework's own tracer + reverse pass.

Reference behaviour: Paddle's imperative tracer records one grad node per op and
``Tensor.backward`` runs a dependency-counted reverse sweep that accumulates into
leaf ``.grad`` (paddle/fluid/imperative/{tracer,engine}.cc in later Paddle; the 0.14
snapshot differentiates Programs instead: python/paddle/fluid/backward.py:315-469,
which the Fluid side of this package mirrors).  Here:

* ``Tensor`` is the framework's tensor handle.  Its storage and kernels are the
  PyTorch-ROCm tensor it wraps (``torch.Tensor`` subclass); every op on it enters
  :meth:`Tensor.__torch_function__`, which runs the op with torch autograd OFF and,
  when an input needs a gradient, records a :class:`GradNode` holding the op's
  explicit backward (``autograd/rules.py``: hand-written VJPs, dispatched to the
  HIP kernels on the GPU where the op library has them; fused ops record their own
  ``Function.backward`` through :func:`record_function`).
* :func:`backward` walks the reachable graph once to count dependencies, then runs
  nodes in topological order, summing gradients per node output and into leaf
  ``.grad`` (fp32/bf16 as the leaf), firing a leaf's grad-ready hooks after its LAST
  contribution in this sweep (DataParallel bucket readiness).
* torch.autograd is never called for a recorded op.  Ops with no rule use the
  last-resort ``fallback`` node (re-run under torch autograd and differentiated by
  ``torch.autograd.grad``); every such op name is logged in :data:`FALLBACK_OPS` so
  tests can assert that a model family never takes it.
"""
from __future__ import annotations

import contextlib
import functools
import threading

import torch
from torch._C import DisableTorchFunctionSubclass

from ..utils import strict as _strict

_TLS = threading.local()
FALLBACK_OPS: dict = {}      # op name -> count of fallback nodes recorded
_RULES: dict = {}             # torch callable -> rule(out, *args, **kwargs) -> (inputs, backward)
_NONDIFF: set = set()         # callables whose float outputs never carry a gradient
_PASS: set = set()            # callables returned raw (no wrap, no record)
_INPLACE: dict = {}           # in-place callable -> out-of-place callable
_FWD_RULES: dict = {}         # callable -> rule(*args, **kwargs) -> (out, inputs, backward)


# ---------------------------------------------------------------------------- grad mode
def is_grad_enabled() -> bool:
    return getattr(_TLS, "grad", True) and torch.is_grad_enabled()


class _GradMode(contextlib.ContextDecorator):
    def __init__(self, mode: bool):
        self.mode = mode

    def __enter__(self):
        self.prev = (getattr(_TLS, "grad", True), torch.is_grad_enabled())
        _TLS.grad = self.mode
        torch.set_grad_enabled(self.mode)

    def __exit__(self, *exc):
        _TLS.grad, tg = self.prev
        torch.set_grad_enabled(tg)
        return False


def no_grad(func=None):
    """``paddle.no_grad``: context manager and decorator (disables recording)."""
    if callable(func):
        return _GradMode(False)(func)
    return _GradMode(False)


def enable_grad():
    return _GradMode(True)


def set_grad_enabled(mode: bool):
    return _GradMode(bool(mode))


# ---------------------------------------------------------------------------- graph
class GradNode:
    """One recorded op.  ``edges[i]`` is where the gradient of differentiable input i
    goes: ``(node, output_index)``, ``(None, leaf_tensor)`` or ``None``."""

    __slots__ = ("name", "backward", "edges", "nout", "out_meta", "accum", "prev")

    def __init__(self, name, backward, edges, nout, out_meta):
        self.name = name
        self.backward = backward
        self.edges = edges
        self.nout = nout
        self.out_meta = out_meta  # (shape, dtype, device) per output, to materialise zero grads
        # accum: the backward may sum an input gradient INTO the gradient the engine
        # already holds for that input (``prev[i]``, offered only when its producer
        # marked it exclusively owned: ``_pa_acc_ok``) and return that same tensor --
        # e.g. a conv's dX accumulated onto the residual branch's gradient in the GEMM
        # epilogue instead of a separate add pass
        self.accum = False
        self.prev = None

    def __repr__(self):
        return f"<GradNode {self.name}>"


def _raw(t):
    return t.as_subclass(torch.Tensor) if isinstance(t, Tensor) else t


def _is_float(t):
    return t.is_floating_point() or t.is_complex()


def _edge(t):
    """Gradient destination of tensor input ``t`` (called with subclass dispatch off)."""
    if not isinstance(t, torch.Tensor):
        return None
    node = t.__dict__.get("_pa_node") if hasattr(t, "__dict__") else None
    if node is not None:
        return (node, t.__dict__["_pa_idx"])
    if t.requires_grad and _is_float(t):
        # a leaf, or a raw torch tensor carrying torch-autograd history (interop with
        # torch-native code upstream: its gradient is handed to torch.autograd)
        return (None, t)
    return None


def tracked(t) -> bool:
    if not isinstance(t, torch.Tensor):
        return False
    with DisableTorchFunctionSubclass():
        return _edge(t) is not None


def _record(name, backward, inputs, outputs):
    """Attach a grad node for ``outputs`` (tensors; non-float ones are skipped) whose
    backward maps the output grads to grads of ``inputs``."""
    edges = [_edge(a) for a in inputs]
    if not any(e is not None for e in edges):
        return None
    meta = [(o.shape, o.dtype, o.device) if isinstance(o, torch.Tensor) else None for o in outputs]
    node = GradNode(name, backward, edges, len(outputs), meta)
    for i, o in enumerate(outputs):
        if isinstance(o, torch.Tensor) and _is_float(o):
            o.__dict__["_pa_node"] = node
            o.__dict__["_pa_idx"] = i
    return node


def _flat_tensors(obj, out):
    if isinstance(obj, torch.Tensor):
        out.append(obj)
    elif isinstance(obj, (list, tuple)):
        for x in obj:
            _flat_tensors(x, out)
    return out


def _wrap(obj):
    if isinstance(obj, torch.Tensor):
        return obj if isinstance(obj, Tensor) else obj.as_subclass(Tensor)
    if isinstance(obj, (tuple, list)) and any(isinstance(x, torch.Tensor) for x in obj):
        vals = [_wrap(x) for x in obj]
        try:
            return type(obj)(vals)  # list, tuple, torch.return_types.* structseqs
        except TypeError:
            return tuple(vals)
    return obj


def _fname(func):
    return getattr(func, "__qualname__", None) or getattr(func, "__name__", None) or repr(func)


def _fallback(func, args, kwargs, out):
    """Last resort for an op with no rule: keep a torch-autograd replay of it."""
    name = _fname(func)
    FALLBACK_OPS[name] = FALLBACK_OPS.get(name, 0) + 1
    ins = [a for a in _flat_tensors(list(args) + list(kwargs.values()), []) if _is_float(a)]

    def bwd(*gouts):
        with torch.enable_grad():
            det = {id(a): a.detach().requires_grad_(True) for a in ins}

            def sub(x):
                if isinstance(x, torch.Tensor) and id(x) in det:
                    return det[id(x)]
                if isinstance(x, (list, tuple)):
                    return type(x)(sub(y) for y in x)
                return x

            r = func(*sub(list(args)), **{k: sub(v) for k, v in kwargs.items()})
            outs = _flat_tensors(r, [])
            pairs = [(o, g) for o, g in zip(outs, gouts) if g is not None and o.requires_grad]
            if not pairs:
                return tuple(None for _ in ins)
            gs = torch.autograd.grad([p[0] for p in pairs], [det[id(a)] for a in ins], [p[1] for p in pairs],
                                     allow_unused=True)
        return gs

    return ins, bwd


# ---------------------------------------------------------------------------- Tensor
class Tensor(torch.Tensor):
    """The framework tensor (``paddle.Tensor``).  ``stop_gradient`` is Paddle's flag
    (True by default for data, False for trainable parameters)."""

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if not _strict.inside() and _strict.watching():
            # framework region: covered ATen ops run on the HIP kernels
            # (ops/aten_native.py); the rest are counted / refused in strict mode.
            # Inside a layer's forward the layer's region is already active.
            with _strict.region("eager:" + _fname(func)):
                return cls._torch_function_impl(func, args, kwargs)
        return cls._torch_function_impl(func, args, kwargs)

    @classmethod
    def _torch_function_impl(cls, func, args, kwargs):
        with DisableTorchFunctionSubclass():
            if func in _PASS:
                return func(*args, **kwargs)
            rec = is_grad_enabled() and _tape_idle() and func not in _NONDIFF
            if rec:
                ins = _flat_tensors(list(args) + list(kwargs.values()), [])
                rec = any(_edge(a) is not None for a in ins)
            if not rec:
                prev = torch.is_grad_enabled()
                torch._C._set_grad_enabled(False)
                try:
                    out = func(*args, **kwargs)
                finally:
                    torch._C._set_grad_enabled(prev)
                return _wrap(out)
            return _dispatch_recorded(func, args, kwargs)

    # --------------------------------------------------------------- Paddle surface
    def backward(self, grad_tensor=None, retain_graph=False):
        backward([self], [grad_tensor], retain_graph=retain_graph)

    @property
    def stop_gradient(self):
        with DisableTorchFunctionSubclass():
            return _edge(self) is None

    @stop_gradient.setter
    def stop_gradient(self, v):
        with DisableTorchFunctionSubclass():
            if "_pa_node" in self.__dict__:  # an op output: stopping cuts it from the graph
                if v:
                    self.__dict__.pop("_pa_node", None)
            else:
                self.requires_grad_(not v)

    def register_hook(self, hook):
        """Gradient hook: ``hook(grad) -> grad or None`` on the gradient flowing into
        this tensor (leaf: before accumulation)."""
        hooks = self.__dict__.setdefault("_pa_hooks", [])
        hooks.append(hook)
        return _HookHandle(hooks, hook)

    def clear_gradient(self, set_to_zero=True):
        with DisableTorchFunctionSubclass():
            if self.grad is not None:
                if set_to_zero:
                    self.grad.zero_()
                else:
                    self.grad = None

    clear_grad = clear_gradient

    def gradient(self):
        with DisableTorchFunctionSubclass():
            return None if self.grad is None else self.grad.detach().cpu().numpy()

    def astype(self, dtype):
        from ..tensor_api import _dtype

        return self.to(_dtype(dtype))

    @property
    def place(self):
        with DisableTorchFunctionSubclass():
            return str(self.device).replace("cuda", "gpu")

    @property
    def grad_node(self):
        return self.__dict__.get("_pa_node")

    def __repr__(self, *, tensor_contents=None):
        with DisableTorchFunctionSubclass():
            body = torch.Tensor.__repr__(self)
        return f"Tensor(stop_gradient={self.stop_gradient}, {body[len('tensor('):]}" if body.startswith(
            "tensor(") else body

    def __reduce_ex__(self, proto):
        with DisableTorchFunctionSubclass():
            return (_rebuild, (torch.Tensor.__reduce_ex__(self.detach(), proto), self.stop_gradient))


def _rebuild(red, stop_gradient):
    fn, args = red[0], red[1]
    t = fn(*args).as_subclass(Tensor)
    if not stop_gradient:
        t.requires_grad_(True)
    return t


class _HookHandle:
    def __init__(self, lst, h):
        self.lst, self.h = lst, h

    def remove(self):
        if self.h in self.lst:
            self.lst.remove(self.h)


def _tape_idle():
    from . import tape

    return tape.current() is None


def _dispatch_recorded(func, args, kwargs):
    """Run ``func`` (subclass dispatch already off) and record its backward."""
    inplace = _INPLACE.get(func)
    if inplace is not None or func is torch.Tensor.__setitem__:
        return _dispatch_inplace(func, inplace, args, kwargs)
    prev = torch.is_grad_enabled()
    torch._C._set_grad_enabled(False)
    try:
        fwd = _FWD_RULES.get(func)
        res = fwd(*args, **kwargs) if fwd is not None else None
        if res is not None:
            out, ins, bwd = res
        else:
            out = func(*args, **kwargs)
    finally:
        torch._C._set_grad_enabled(prev)
    if not any(_is_float(o) for o in _flat_tensors(out, [])):
        return _wrap(out)
    if isinstance(out, torch.Tensor) and any(out is a for a in _flat_tensors(list(args) + list(kwargs.values()), [])):
        return out  # the op returned its input (e.g. .float() of an fp32 tensor): identity, nothing to record
    out = _wrap(out)
    outs = _flat_tensors(out, [])
    if res is None:
        rule = _RULES.get(func)
        rkw = {k: v for k, v in kwargs.items() if k != "out"} if "out" in kwargs else kwargs
        r = rule(out, *args, **rkw) if rule is not None else None
        ins, bwd = r if r is not None else _fallback(func, args, kwargs, out)
    _record(_fname(func), bwd, ins, outs)
    return out


def _dispatch_inplace(func, outofplace, args, kwargs):
    """In-place op on a tracked tensor: computed out of place (recorded), then copied
    into the target, which takes over the new node (Paddle's inplace version bump)."""
    tgt = args[0]
    if tgt.is_leaf and tgt.requires_grad:
        raise RuntimeError(f"in-place op {_fname(func)} on a leaf Tensor that requires grad "
                           "(stop_gradient=False); use the out-of-place op or paddle.no_grad()")
    if func is torch.Tensor.__setitem__:
        from .rules import setitem_outofplace

        res = setitem_outofplace(*args)
    else:
        res = _dispatch_recorded(outofplace, args, kwargs)
    prev = torch.is_grad_enabled()
    torch._C._set_grad_enabled(False)
    try:
        torch.Tensor.copy_(tgt, res)
    finally:
        torch._C._set_grad_enabled(prev)
    node = res.__dict__.get("_pa_node") if isinstance(res, torch.Tensor) else None
    if node is not None:
        if not isinstance(tgt, Tensor):
            # a raw torch tensor written in place from a tracked value becomes a framework
            # Tensor (same object), so later ops on it are still recorded
            tgt.__class__ = Tensor
        tgt.__dict__["_pa_node"] = node
        tgt.__dict__["_pa_idx"] = res.__dict__["_pa_idx"]
    else:
        tgt.__dict__.pop("_pa_node", None)
    return None if func is torch.Tensor.__setitem__ else tgt


def record_function(fn, args):
    """Eager-mode application of a fused op ``fn`` (a ``torch.autograd.Function``
    with hand-written forward / backward): forward with torch autograd off, one grad
    node whose backward is ``fn.backward``.  Returns None when no input is tracked."""
    from .tape import _Ctx

    with DisableTorchFunctionSubclass():
        edges = [_edge(a) for a in args]
        if not any(e is not None for e in edges):
            return None
        ctx = _Ctx(tuple(e is not None for e in edges))
        prev = torch.is_grad_enabled()
        torch._C._set_grad_enabled(False)
        try:
            out = fn.forward(ctx, *[_raw(a) for a in args])
        finally:
            torch._C._set_grad_enabled(prev)
        single = not isinstance(out, tuple)
        out = _wrap(out)
        outs = [out] if single else list(out)

        holder = []

        def bwd(*gouts):
            # hand-written backward kernels index their gradient inputs densely
            gouts = [g.contiguous() if isinstance(g, torch.Tensor) else g for g in gouts]
            ctx.grad_prev = holder[0].prev if holder else None
            r = fn.backward(ctx, *gouts)
            ctx.grad_prev = None
            return r if isinstance(r, tuple) else (r,)

        node = _record(getattr(fn, "__name__", "fused"), bwd, list(args), outs)
        if node is not None:
            node.accum = True
            holder.append(node)
        return out


# ---------------------------------------------------------------------------- backward
def _accumulate(a, b):
    if a is None:
        return b
    if b is None:
        return a
    return a + b


def backward(tensors, grad_tensors=None, retain_graph=False):
    """Reverse sweep from ``tensors`` (``paddle.autograd.backward``)."""
    with DisableTorchFunctionSubclass():
        _backward(list(tensors), list(grad_tensors or [None] * len(tensors)), retain_graph)


def in_backward() -> bool:
    return getattr(_TLS, "callbacks", None) is not None


def queue_callback(fn):
    """Run ``fn()`` when the current eager backward sweep ends (torch's
    ``queue_callback`` contract, for DataParallel's final bucket wait)."""
    cbs = getattr(_TLS, "callbacks", None)
    if cbs is None:
        raise RuntimeError("queue_callback outside of an eager backward")
    cbs.append(fn)


def add_grad_ready_hook(p, fn):
    """``fn(p)`` after ``p``'s LAST gradient contribution of a sweep has been
    accumulated into ``p.grad`` (post-accumulate-grad hook)."""
    p.__dict__.setdefault("_pa_grad_ready_hooks", []).append(fn)


def _backward(roots, grads, retain_graph):
    from . import tape as _tape

    _tape.run_before_backward()  # e.g. an optimizer update still running on a side stream
    if not _strict.inside() and _strict.watching():
        with _strict.region("eager:backward"):
            return _backward_impl(roots, grads, retain_graph)
    return _backward_impl(roots, grads, retain_graph)


def _backward_impl(roots, grads, retain_graph):
    prev = torch.is_grad_enabled()
    torch._C._set_grad_enabled(False)
    outer = getattr(_TLS, "callbacks", None)
    _TLS.callbacks = []
    try:
        buffers = {}   # node -> list of grads per output
        deps = {}      # node -> pending consumer count
        leaf_uses = {}  # id(leaf) -> remaining contributions
        leaves = {}
        start = []
        for t, g in zip(roots, grads):
            e = _edge(t)
            if e is None:
                raise RuntimeError("backward() on a Tensor with stop_gradient=True (nothing requires grad)")
            if g is None:
                if t.numel() != 1:
                    raise RuntimeError("backward() of a non-scalar Tensor needs grad_tensor")
                g = torch.ones_like(_raw(t))
            g = _raw(g)
            node, idx = e
            if node is None:  # backward on a leaf itself
                _leaf_add(idx, g)
                continue
            buf = buffers.setdefault(node, [None] * node.nout)
            buf[idx] = _accumulate(buf[idx], g)
            start.append(node)
        # dependency counts over the reachable graph
        seen = set()
        stack = list(dict.fromkeys(start))
        for n in stack:
            seen.add(n)
        while stack:
            n = stack.pop()
            for e in n.edges:
                if e is None:
                    continue
                child, tgt = e
                if child is None:
                    leaf_uses[id(tgt)] = leaf_uses.get(id(tgt), 0) + 1
                    leaves[id(tgt)] = tgt
                    continue
                deps[child] = deps.get(child, 0) + 1
                if child not in seen:
                    seen.add(child)
                    stack.append(child)
        ready = [n for n in dict.fromkeys(start) if deps.get(n, 0) == 0]
        pending = {}  # id(leaf) -> grad summed over this sweep
        torch_roots = []
        while ready:
            n = ready.pop()
            gouts = buffers.pop(n, None) or [None] * n.nout
            if n.backward is None:
                raise RuntimeError(f"grad node {n.name} was already freed: call backward(retain_graph=True) "
                                   "to differentiate a graph twice")
            if any(g is not None for g in gouts):
                gouts = [g if g is not None or m is None or not _is_float_dtype(m[1])
                         else torch.zeros(m[0], dtype=m[1], device=m[2]) for g, m in zip(gouts, n.out_meta)]
                if n.accum and _ACCUM_INTO[0]:
                    n.prev = _prev_grads(n, buffers)
                gins = n.backward(*gouts)
                n.prev = None
                if not isinstance(gins, (tuple, list)):
                    gins = (gins,)
            else:
                gins = (None,) * len(n.edges)
            if not retain_graph:
                n.backward = None
            for e, g in zip(n.edges, list(gins) + [None] * (len(n.edges) - len(gins))):
                if e is None:
                    continue
                child, tgt = e
                if child is None:
                    if g is not None:
                        pending[id(tgt)] = _accumulate(pending.get(id(tgt)), g)
                    leaf_uses[id(tgt)] -= 1
                    if leaf_uses[id(tgt)] == 0:
                        _leaf_add(tgt, pending.pop(id(tgt), None), torch_roots)
                    continue
                if g is not None:
                    buf = buffers.setdefault(child, [None] * child.nout)
                    cur = buf[tgt]
                    buf[tgt] = g if g is cur else _accumulate(cur, g)  # `is`: summed in place by the backward
                deps[child] -= 1
                if deps[child] == 0:
                    ready.append(child)
        if torch_roots:
            torch.autograd.backward([t for t, _ in torch_roots], [g for _, g in torch_roots])
        cbs = _TLS.callbacks
        _TLS.callbacks = outer
        for cb in cbs:
            cb()
    finally:
        _TLS.callbacks = outer
        torch._C._set_grad_enabled(prev)


_ACCUM_INTO = [__import__("os").environ.get("FLAGS_eager_accumulate_into", "1") != "0"]


def _prev_grads(n, buffers):
    """Per input edge of ``n``: the gradient already accumulated for that input when
    its producer marked it exclusively owned (``_pa_acc_ok``), else None."""
    out = []
    for e in n.edges:
        g = None
        if e is not None and e[0] is not None:
            b = buffers.get(e[0])
            if b is not None:
                g = b[e[1]]
                if g is not None and not getattr(g, "_pa_acc_ok", False):
                    g = None
        out.append(g)
    return out


def _is_float_dtype(dt):
    return dt.is_floating_point or dt.is_complex


def _leaf_add(leaf, g, torch_roots=None):
    if leaf.grad_fn is not None:  # torch-autograd history upstream: one torch backward per sweep
        if g is not None and torch_roots is not None:
            torch_roots.append((leaf, g.to(leaf.dtype)))
        return
    if g is not None:
        for h in leaf.__dict__.get("_pa_hooks", ()):
            r = h(_wrap(g))
            if r is not None:
                g = _raw(r)
        if g.shape != leaf.shape:
            g = g.sum_to_size(leaf.shape)
        if g.dtype != leaf.dtype:
            g = g.to(leaf.dtype)
        if leaf.grad is None:
            leaf.grad = g.as_subclass(Tensor) if not isinstance(g, Tensor) else g
        elif leaf.grad.is_cuda:
            from ..ops import oplib

            with DisableTorchFunctionSubclass():
                oplib.add_(leaf.grad, g)  # direct kernel launch (no dispatch-mode hop)
        else:
            leaf.grad.add_(g)
    for hook in leaf.__dict__.get("_pa_grad_ready_hooks", ()):
        hook(leaf)


def grad(outputs, inputs, grad_outputs=None, retain_graph=None, create_graph=False, allow_unused=False):
    """``paddle.grad``: gradients of ``outputs`` w.r.t. ``inputs`` without touching
    ``.grad`` (create_graph is not supported: no higher-order rules)."""
    if create_graph:
        raise NotImplementedError("paddle.grad(create_graph=True): higher-order gradients are not supported")
    outputs = [outputs] if isinstance(outputs, torch.Tensor) else list(outputs)
    single = isinstance(inputs, torch.Tensor)
    inputs = [inputs] if single else list(inputs)
    saved = {}
    with DisableTorchFunctionSubclass():
        for x in inputs:
            leaf = "_pa_node" not in x.__dict__
            saved[id(x)] = (x.grad if leaf else None, x.__dict__.get("_pa_hooks"))
            if leaf:
                x.grad = None
        cap = {}
        for x in inputs:
            if "_pa_node" in x.__dict__:  # a non-leaf: capture the gradient flowing into it
                node, idx = x.__dict__["_pa_node"], x.__dict__["_pa_idx"]
                cap[id(x)] = (node, idx)
    res = []
    if cap:
        # gradient w.r.t. intermediate tensors: hook the producing node's output slot
        got = {}

        def make(node, idx, key):
            orig = node.backward

            def wrapped(*gouts):
                got[key] = gouts[idx]
                return orig(*gouts)

            return wrapped

        originals = {}
        for x in inputs:
            if id(x) in cap:
                node, idx = cap[id(x)]
                originals.setdefault(node, node.backward)
                node.backward = make(node, idx, id(x))
        backward(outputs, grad_outputs, retain_graph=True if retain_graph is None else retain_graph)
        for node, orig in originals.items():
            if node.backward is not None:
                node.backward = orig
    else:
        backward(outputs, grad_outputs, retain_graph=bool(retain_graph))
    with DisableTorchFunctionSubclass():
        for x in inputs:
            if id(x) in cap:
                g = got.get(id(x)) if cap else None
            else:
                g = x.grad
                x.grad = saved[id(x)][0]
            if g is None and not allow_unused:
                raise RuntimeError("paddle.grad: an input is not reachable from the outputs (allow_unused=True)")
            res.append(None if g is None else _wrap(g))
    return res[0] if single and len(res) == 1 else res


# ---------------------------------------------------------------------------- registry
def register(*funcs):
    """Decorator: ``rule(out, *args, **kwargs) -> (inputs, backward)`` for ``funcs``;
    ``backward(*grad_outputs)`` returns one gradient (or None) per entry of ``inputs``."""

    def deco(rule):
        for f in funcs:
            _RULES[f] = rule
        return rule

    return deco


def nondiff(*funcs):
    _NONDIFF.update(funcs)


def passthrough(*funcs):
    _PASS.update(funcs)


def inplace(mapping):
    _INPLACE.update(mapping)


def to_tensor_handle(t, stop_gradient=True):
    """Wrap a torch tensor as a framework Tensor (no copy)."""
    if not isinstance(t, torch.Tensor):
        raise TypeError(type(t))
    out = t if isinstance(t, Tensor) else t.as_subclass(Tensor)
    if not stop_gradient:
        out.requires_grad_(True)
    return out


def wraps_outputs(fn):
    """Decorator for ``paddle.*`` creation / math functions: torch tensors they return
    become framework Tensors."""

    @functools.wraps(fn)
    def w(*a, **k):
        return _wrap(fn(*a, **k))

    return w

from . import rules as _rules  # noqa: E402,F401  (registers the backward rules)
