"""FP8 (OCP e4m3fn) weight GEMMs for MI355X.

gfx950 MFMA runs fp8 x fp8 -> fp32 at 2x the bf16 rate (``v_mfma_f32_32x32x64_f8f6f4``
/ the non-scaled 32x32x16 fp8 forms).  ``fp8_linear`` keeps a bf16/fp32 master
weight (the optimizer updates it), caches its e4m3 copy + per-tensor scale keyed
on the weight's version counter, quantises the activation with a dynamic
per-tensor amax scale and runs the FORWARD GEMM in fp8 through hipBLASLt
(``torch._scaled_mm``); the backward GEMMs run in bf16 against the master weight
(straight-through estimator), the usual recipe for fp8 training of MoE experts.

On CPU (tests) or where the fp8 GEMM is unavailable the same quantise/dequantise
numerics are emulated in fp32, so results match the device path to fp8 rounding.
"""
from __future__ import annotations

import torch

E4M3_MAX = 448.0
_FP8 = getattr(torch, "float8_e4m3fn", None)
_scaled_mm_ok = {}


def quantize(x, amax=None):
    """Per-tensor e4m3 quantisation: returns (fp8 tensor, fp32 scale) with x ~= q * scale."""
    a = x.detach().abs().amax().float() if amax is None else amax
    scale = torch.clamp(a, min=1e-12) / E4M3_MAX
    q = (x.float() / scale).clamp(-E4M3_MAX, E4M3_MAX).to(_FP8)
    return q, scale


def _can_scaled_mm(dev):
    if dev.type != "cuda" or _FP8 is None or not hasattr(torch, "_scaled_mm"):
        return False
    key = dev.index or 0
    if key not in _scaled_mm_ok:
        try:
            a = torch.zeros(32, 32, device=dev, dtype=_FP8)
            b = torch.zeros(32, 32, device=dev, dtype=_FP8).t()
            one = torch.ones((), device=dev)
            torch._scaled_mm(a, b, scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
            _scaled_mm_ok[key] = True
        except Exception:  # noqa: BLE001
            _scaled_mm_ok[key] = False
    return _scaled_mm_ok[key]


class _WeightCache:
    def __init__(self):
        self.version = -1
        self.q = self.scale = None


def _weight_fp8(w, cache):
    v = w._version
    if cache.version != v or cache.q is None:
        # [in, out] master -> column-major [out, in]^T view for _scaled_mm's B operand
        cache.q, cache.scale = quantize(w.detach().t().contiguous())
        cache.version = v
    return cache.q, cache.scale


class _FP8LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, cache):
        x2 = x.reshape(-1, x.shape[-1])
        wq, ws = _weight_fp8(w, cache)         # wq: [out, in] e4m3
        xq, xs = quantize(x2)
        if _can_scaled_mm(x.device) and x2.shape[0] % 16 == 0 and x2.shape[1] % 16 == 0 and wq.shape[0] % 16 == 0:
            y = torch._scaled_mm(xq, wq.t(), scale_a=xs, scale_b=ws, out_dtype=torch.bfloat16)
            y = y.to(x.dtype)
        else:
            y = ((xq.float() * xs) @ (wq.float() * ws).t()).to(x.dtype)
        if b is not None:
            y = y + b
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        return y.reshape(*x.shape[:-1], w.shape[1])

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        g2 = g.reshape(-1, g.shape[-1])
        x2 = x.reshape(-1, x.shape[-1])
        dx = (g2 @ w.t().to(g2.dtype)).reshape(x.shape)
        dw = (x2.t().to(g2.dtype) @ g2).to(w.dtype)
        db = g2.sum(0).to(w.dtype) if ctx.has_b else None
        return dx, dw, db, None


def fp8_linear(x, weight, bias=None, cache=None):
    """``x @ weight (+ bias)`` with ``weight`` [in, out] (Paddle layout) run as an fp8 GEMM."""
    if cache is None:
        cache = getattr(weight, "_pa_fp8_cache", None)
        if cache is None:
            cache = _WeightCache()
            try:
                weight._pa_fp8_cache = cache
            except Exception:  # noqa: BLE001
                pass
    return _FP8LinearFn.apply(x, weight, bias, cache)
