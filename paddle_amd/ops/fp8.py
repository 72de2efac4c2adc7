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
from ..autograd import tape as _tape  # noqa: E402

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
    return _tape.apply(_FP8LinearFn, x, weight, bias, cache)


# ---------------------------------------------------------------- native fp8 GEMM
# gemm.hip ``pa_gemm_f8``: block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 (2x the
# bf16 MFMA rate), both operands K-major e4m3, fp32 per-row (A) / per-column (B)
# scales applied in the epilogue.  fp8.hip quantises rows (activations, weights
# read as stored) or transposes + quantises columns (Paddle [in, out] weights).


def quant_rows(x):
    """x [R, K] bf16 (K % 16 == 0) -> (q [R, K] e4m3, scale [R] fp32), x ~= q * scale[:, None]."""
    from . import _native as N

    R, K = x.shape
    q = torch.empty(R, K, dtype=_FP8, device=x.device)
    s = torch.empty(R, dtype=torch.float32, device=x.device)
    N.call("pa_quant_rows_f8", N.ptr(x), x.stride(0), N.ptr(q), K, N.ptr(s), R, K, N.stream())
    return q, s


def quant_cols_t(w):
    """w [G, K, N] bf16 -> (qt [G, N, K] e4m3, scale [G, N]): per-output-channel scales."""
    from . import _native as N

    w = w.contiguous()
    G, K, Nn = w.shape
    qt = torch.empty(G, Nn, K, dtype=_FP8, device=w.device)
    s = torch.empty(G, Nn, dtype=torch.float32, device=w.device)
    N.call("pa_quant_cols_t_f8", N.ptr(w), N.ptr(qt), N.ptr(s), G, K, Nn, N.stream())
    return qt, s


def gemm_f8(aq, sa, bq, sb, M, Nn, K, *, out, batch=1, sB=0, grp=None, grp_mode=0, alpha=1.0, accumulate=False):
    """out[m, n] (=|+=) alpha * sa[m] * sb[g, n] * sum_k aq[m, k] bq[g][n, k]."""
    from . import _native as N

    rc = N.lib().pa_gemm_f8(int(out.dtype == torch.float32), N.ptr(aq), N.ptr(bq), N.ptr(out), N.ptr(sa), N.ptr(sb),
                            M, Nn, K, aq.stride(0), bq.stride(-2), out.stride(0), sB, 0, batch, float(alpha),
                            int(accumulate), N.ptr(grp), int(grp_mode), N.stream())
    if rc != 0:
        raise RuntimeError(f"pa_gemm_f8 failed (rc={rc}) M={M} N={Nn} K={K}")
    return out


class VersionedCache:
    """Holds derived tensors of a parameter (fp8 copies), rebuilt when the weight
    changes: its version counter or the optimizer weight epoch moves."""

    def __init__(self, build):
        self.build = build
        self.version = None
        self.value = None

    def get(self, w):
        from .fused import _WEIGHT_EPOCH  # bumped by optimizers that write through raw pointers

        v = (_WEIGHT_EPOCH[0], w.data_ptr(), w._version)
        if self.version != v:
            self.value = self.build(w.detach())
            self.version = v
        return self.value
