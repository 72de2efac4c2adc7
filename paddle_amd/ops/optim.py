"""Fused optimizer kernels over flat buffers (GPU: gfx950 kernels; CPU: torch math).

Parity: reference adam / momentum / sgd ops (paddle/fluid/operators/adam_op.h:35-321,
momentum_op.cu:67, sgd_op.cu:73).  The GPU path updates a whole flat parameter
shard in one launch and writes the bf16 model copy in the same pass.
"""
from __future__ import annotations

import torch

from . import _native as N
from . import fused as _fused


def adamw_flat(param, grad, m, v, *, lr, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0,
               step=1, param_out=None, decay_end=None, grad_scale=1.0, lr_tensor=None,
               beta1_pow=None, beta2_pow=None, grad_scale_tensor=None, lr_t_eps=False):
    """In-place AdamW on fp32 ``param`` (flat, contiguous) with fp32 moments.

    ``decay_end``: elements with index < decay_end get decoupled weight decay
    (the flat layout puts all decayed params first).  ``param_out``: optional
    bf16/fp32 copy written in the same pass.  ``lr_tensor``/``beta*_pow``:
    device scalars (static-graph adam op semantics, no host sync).  ``lr_t_eps``:
    Kingma/Paddle epsilon placement (adam_op.h): p -= lr*sqrt(1-b2^t)/(1-b1^t) * m/(sqrt(v)+eps).
    """
    n = param.numel()
    if decay_end is None:
        decay_end = n
    bc1 = 1.0 - beta1 ** step
    bc2 = 1.0 - beta2 ** step
    if param.is_cuda:
        _fused.bump_weight_epoch()
        N.call("pa_adamw", N.dt(grad), (N.dt(param_out) if param_out is not None else -1), N.ptr(param),
               N.ptr(grad), N.ptr(m), N.ptr(v), N.ptr(param_out), n, float(lr), N.ptr(lr_tensor),
               float(beta1), float(beta2), float(eps), float(weight_decay), float(bc1), float(bc2),
               N.ptr(beta1_pow), N.ptr(beta2_pow), int(decay_end), float(grad_scale),
               N.ptr(grad_scale_tensor), int(lr_t_eps), N.stream())
        return param
    lr_ = float(lr_tensor.reshape(-1)[0]) if lr_tensor is not None else lr
    if beta1_pow is not None:
        bc1 = 1.0 - float(beta1_pow.reshape(-1)[0])
        bc2 = 1.0 - float(beta2_pow.reshape(-1)[0])
    gs = grad_scale * (float(grad_scale_tensor.reshape(-1)[0]) if grad_scale_tensor is not None else 1.0)
    g = grad.float() * gs
    m.mul_(beta1).add_(g, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    if weight_decay:
        idx = torch.arange(n, device=param.device) < decay_end
        param.mul_(torch.where(idx, 1 - lr_ * weight_decay, 1.0))
    e = eps / (bc2 ** 0.5) if lr_t_eps else eps
    param.addcdiv_(m / bc1, (v / bc2).sqrt_().add_(e), value=-lr_)
    if param_out is not None:
        param_out.copy_(param)
    return param


def momentum_flat(param, grad, velocity=None, *, lr, mu=0.9, nesterov=False, weight_decay=0.0,
                  grad_scale=1.0, lr_tensor=None):
    n = param.numel()
    if param.is_cuda:
        _fused.bump_weight_epoch()
        if param.dtype not in (torch.float32, torch.bfloat16) or not param.is_contiguous():
            raise TypeError(f"momentum_flat: contiguous fp32 / bf16 parameter required, got {param.dtype}")
        N.call("pa_momentum_p", N.dt(grad), N.dt(param), N.ptr(param), N.ptr(grad), N.ptr(velocity), n,
               float(lr), N.ptr(lr_tensor), float(mu), int(nesterov), float(weight_decay), float(grad_scale),
               N.stream())
        return param
    lr_ = float(lr_tensor.reshape(-1)[0]) if lr_tensor is not None else lr
    pf = param.float()
    g = grad.float() * grad_scale + weight_decay * pf
    if velocity is None:
        param.copy_(pf - lr_ * g)
        return param
    velocity.mul_(mu).add_(g)
    param.copy_(pf - (lr_ * (g + mu * velocity) if nesterov else lr_ * velocity))
    return param


class MomentumMulti:
    """Multi-tensor Momentum (``pa_momentum_multi``): one launch updates every
    parameter.  The per-tensor descriptor table lives on the device and is re-uploaded
    only when a pointer changes (steady-state training re-uses the caching
    allocator's grad addresses); uploads go through two pinned host buffers, each
    re-used only after the copy that read it has completed (event)."""

    _DT = None

    def __init__(self):
        self._key = None
        self._dev = None
        self._chunks = 0
        self._nt = 0
        self._pinned = [None, None]
        self._events = [None, None]
        self._flip = 0

    @classmethod
    def _dtype(cls):
        if cls._DT is None:
            import numpy as np

            cls._DT = np.dtype([("t", "<u8"), ("out", "<u8"), ("g", "<u8"), ("vel", "<u8"), ("n", "<i8"),
                                ("chunk0", "<i8"), ("wd", "<f4"), ("lr_scale", "<f4"), ("tdt", "<i4"),
                                ("odt", "<i4"), ("gdt", "<i4"), ("pad", "<i4")])
            assert cls._DT.itemsize == int(N.lib().pa_momentum_multi_entry_bytes())
        return cls._DT

    def step(self, entries, *, lr, mu, nesterov=False, grad_scale=1.0, lr_tensor=None):
        """entries: list of (target, out_or_None, grad, velocity, weight_decay, lr_scale);
        target / out fp32 or bf16 contiguous, velocity fp32."""
        if not entries:
            return
        import numpy as np

        _fused.bump_weight_epoch()
        key = tuple((t.data_ptr(), o.data_ptr() if o is not None else 0, g.data_ptr(), v.data_ptr(), t.numel(),
                     N.dt(t), N.dt(o) if o is not None else 0, N.dt(g), float(wd), float(ls))
                    for t, o, g, v, wd, ls in entries)
        if key != self._key:
            chunk = int(N.lib().pa_momentum_multi_chunk())
            arr = np.zeros(len(key), dtype=self._dtype())
            c0 = 0
            for i, (tp, op, gp, vp, n, tdt, odt, gdt, wd, ls) in enumerate(key):
                arr[i] = (tp, op, gp, vp, n, c0, wd, ls, tdt, odt, gdt, 0)
                c0 += (n + chunk - 1) // chunk
            raw = torch.from_numpy(arr.view(np.uint8))
            dev = entries[0][0].device
            if torch.cuda.is_current_stream_capturing():
                # HIP-graph capture (graph-pool gradient addresses): a table of its own,
                # uploaded by a captured copy from a spare pinned buffer set aside by an
                # earlier eager step (no host allocation or event wait inside a capture)
                spares = getattr(self, "_spares", [])
                pin = next((p for p in spares if p.numel() >= raw.numel()), None)
                if pin is None:
                    raise RuntimeError("MomentumMulti: run one eager step before capturing it in a HIP graph")
                spares.remove(pin)
                pin = pin[:raw.numel()]
                pin.copy_(raw)
                d = torch.empty(raw.numel(), dtype=torch.uint8, device=dev)
                d.copy_(pin, non_blocking=True)
                self._graph_tables = getattr(self, "_graph_tables", []) + [(pin, d)]
                N.call("pa_momentum_multi", N.ptr(d), len(key), c0, float(lr), N.ptr(lr_tensor), float(mu),
                       int(nesterov), float(grad_scale), N.stream())
                return
            b = self._flip
            self._flip ^= 1
            if self._events[b] is not None:
                self._events[b].synchronize()
            if self._pinned[b] is None or self._pinned[b].numel() < raw.numel():
                self._pinned[b] = torch.empty(raw.numel(), dtype=torch.uint8, pin_memory=True)
                # pinned buffers for up to two later HIP-graph captures of this step
                self._spares = [torch.empty(raw.numel(), dtype=torch.uint8, pin_memory=True) for _ in range(2)]
            self._pinned[b][:raw.numel()].copy_(raw)
            if self._dev is None or self._dev.numel() < raw.numel():
                self._dev = torch.empty(raw.numel(), dtype=torch.uint8, device=dev)
            self._dev[:raw.numel()].copy_(self._pinned[b][:raw.numel()], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._events[b] = ev
            self._key, self._chunks, self._nt = key, c0, len(key)
        N.call("pa_momentum_multi", N.ptr(self._dev), self._nt, self._chunks, float(lr), N.ptr(lr_tensor),
               float(mu), int(nesterov), float(grad_scale), N.stream())


def sumsq(x, out=None):
    """Sum of squares into a 1-element fp32 tensor (accumulates into ``out``)."""
    if out is None:
        out = torch.zeros(1, dtype=torch.float32, device=x.device)
    if x.is_cuda:
        N.call("pa_sumsq", N.dt(x), N.ptr(x), x.numel(), N.ptr(out), N.stream())
    else:
        out += x.float().pow(2).sum()
    return out
