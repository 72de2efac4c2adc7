"""FP8 (OCP e4m3fn) GEMMs for MI355X on the hand-written gfx950 kernel.

gfx950 runs block-scaled fp8 x fp8 -> fp32 MFMA (``v_mfma_scale_f32_16x16x128_f8f6f4``)
at 2x the bf16 rate; ``gemm.hip``'s ``pa_gemm_f8`` uses it with both operands
K-major e4m3 and fp32 per-row (A) / per-column (B) scales applied in the epilogue.

``fp8_linear`` (dense layers) keeps the bf16 master weight (the optimizer updates
it) and caches two e4m3 images of it, rebuilt when the weight changes: columns
quantised per output channel and transposed ([out, in], forward B operand) and rows
quantised per input channel ([in, out], dgrad B operand).  Forward y = x W and
dgrad dx = dy W^T run in fp8 with per-row dynamic scales of the activation / output
gradient (quantised by fp8.hip); wgrad dW = x^T dy stays bf16 on the same native
GEMM (accumulated in fp32) -- the usual fp8 training recipe.  The grouped expert
GEMMs of the MoE layer use the same kernel (``gemm_f8`` below, grp_mode 1).

On CPU (tests) or for shapes the kernel does not take (K % 16, N % 8) the same
per-row / per-column quantisation is emulated in fp32, so both paths share numerics
up to accumulation order.
"""
from __future__ import annotations

import torch
from ..autograd import tape as _tape  # noqa: E402

E4M3_MAX = 448.0
_FP8 = getattr(torch, "float8_e4m3fn", None)


def quantize(x, amax=None):
    """Per-tensor e4m3 quantisation: returns (fp8 tensor, fp32 scale) with x ~= q * scale."""
    a = x.detach().abs().amax().float() if amax is None else amax
    scale = torch.clamp(a, min=1e-12) / E4M3_MAX
    q = (x.float() / scale).clamp(-E4M3_MAX, E4M3_MAX).to(_FP8)
    return q, scale


def quant_rows_ref(x):
    """Host / fallback twin of fp8.hip's row quantiser: x [R, K] -> (q e4m3, scale [R])."""
    s = torch.clamp(x.detach().float().abs().amax(1), min=1e-12) / E4M3_MAX
    q = (x.float() / s[:, None]).clamp(-E4M3_MAX, E4M3_MAX).to(_FP8)
    return q, s


def _native_ok(x2, w):
    M, K = x2.shape
    N = w.shape[1]
    return (x2.is_cuda and w.is_cuda and x2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and K % 16 == 0 and N % 16 == 0 and M > 0)


class _WeightCache:
    """e4m3 images of one master weight [in, out]: ``fwd`` = per-output-channel
    columns transposed to [out, in]; ``bwd`` = per-input-channel rows [in, out]."""

    def __init__(self):
        self.fwd = VersionedCache(lambda w: tuple(t[0] for t in quant_cols_t(w[None])))
        self.bwd = VersionedCache(lambda w: quant_rows(w.contiguous()))


def _emul(aq, sa, bq, sb):
    """sum_k aq[m, k] bq[n, k] * sa[m] * sb[n] in fp32 (CPU / fallback)."""
    return (aq.float() * sa[:, None]) @ (bq.float() * sb[:, None]).t()


class _FP8LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, cache):
        Kin, N = w.shape
        x2 = x.reshape(-1, Kin)
        M = x2.shape[0]
        native = _native_ok(x2, w)
        if native:
            xq, xs = quant_rows(x2.contiguous())
            wq, ws = cache.fwd.get(w)
            y = gemm_f8(xq, xs, wq, ws, M, N, Kin, out=torch.empty(M, N, dtype=torch.bfloat16, device=x.device))
        else:
            xq, xs = quant_rows_ref(x2)
            wq, ws = quant_rows_ref(w.detach().t())
            y = _emul(xq, xs, wq, ws).to(x.dtype)
        if b is not None:
            y = y + b.to(y.dtype)
        ctx.save_for_backward(x2, w)
        ctx.has_b, ctx.native, ctx.cache, ctx.xshape = b is not None, native, cache, x.shape
        return y.reshape(*x.shape[:-1], N)

    @staticmethod
    def backward(ctx, g):
        x2, w = ctx.saved_tensors
        Kin, N = w.shape
        g2 = g.reshape(-1, N)
        M = g2.shape[0]
        if ctx.native and g2.dtype == torch.bfloat16:
            from . import gemm as G

            gq, gs = quant_rows(g2.contiguous())
            wq, ws = ctx.cache.bwd.get(w)
            dx = gemm_f8(gq, gs, wq, ws, M, Kin, N, out=torch.empty(M, Kin, dtype=torch.bfloat16, device=g.device))
            dw = G.linear_dw(x2.contiguous(), g2.contiguous()).to(w.dtype)
        else:
            gq, gs = quant_rows_ref(g2)
            wq, ws = quant_rows_ref(w.detach())
            dx = _emul(gq, gs, wq, ws).to(g2.dtype)
            dw = (x2.t().float() @ g2.float()).to(w.dtype)
        db = g2.float().sum(0).to(w.dtype) if ctx.has_b else None
        return dx.reshape(ctx.xshape), dw, db, None


def fp8_linear(x, weight, bias=None, cache=None):
    """``x @ weight (+ bias)`` with ``weight`` [in, out] (Paddle layout): forward and
    dgrad on the fp8 MFMA GEMM, wgrad bf16."""
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
