"""Fused hot ops: autograd wrappers over the gfx950 kernels (GPU) and PyTorch
reference math (CPU).

Each op has exactly two kernels, like the reference's CPU/CUDA kernel pair
(SURVEY §2.1 #5): a GPU tensor always runs the hand-written HIP kernel from
``libpaddle_amd_kernels.so`` (loading fails loudly if it is missing) and a CPU
tensor runs the plain PyTorch definition below, which is also the fp32 oracle
the GPU numerics tests compare against.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F

from . import _native as N
from ..autograd import tape as _tape
from . import gemm as _G

# --------------------------------------------------------------------------- utils


def _ws(n: int, device, dtype=torch.float32):
    return torch.empty(n, dtype=dtype, device=device)



def _oplib_fill(t, v):
    from . import oplib

    return oplib.fill_(t, v)


def _fill_native(t, v):
    """t[...] = v (strided views too) on the native elementwise kernel."""
    from . import aten_native as A

    if not (t.is_cuda and t.dtype in A._DT and A._launch(A.U["fill"], t, [], a=float(v), cdt=A._cdt(t.dtype))):
        t.fill_(v)
    return t


def _copy_native(dst, src):
    """dst[...] = src (strided views, same shape) on the native elementwise kernel."""
    from . import aten_native as A

    if not (dst.is_cuda and dst.dtype in A._DT and src.dtype in A._DT
            and A._launch(A.U["copy"], dst, [src], cdt=A._cdt(src.dtype))):
        dst.copy_(src)
    return dst

def _scale_native(x, s):
    """x * s (a new tensor) on the native elementwise kernel (GPU), else torch."""
    if x.is_cuda:
        from . import aten_native as A

        if x.dtype in A._DT:
            out = torch.empty_like(x, memory_format=torch.contiguous_format)
            if A._launch(A.U["affine"], out, [x], a=float(s), b=0.0):
                return out
    return x * s


def _c(t):
    return t if t.is_contiguous() else t.contiguous()


# ====================================================================== RMS / Layer norm


def _norm_ref(x, res, w, b, eps, rms):
    h = x.float() + res.float() if res is not None else x.float()
    if rms:
        rstd = torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + eps)
        y = h * rstd * w.float()
        mean = None
    else:
        mean = h.mean(-1, keepdim=True)
        var = (h - mean).pow(2).mean(-1, keepdim=True)
        rstd = torch.rsqrt(var + eps)
        y = (h - mean) * rstd * w.float()
        if b is not None:
            y = y + b.float()
    return y.to(x.dtype), h.to(x.dtype)


class _NormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, w, b, eps, rms):
        H = x.shape[-1]
        x2 = _c(x).view(-1, H)
        Nr = x2.shape[0]
        dev = x.device
        y = torch.empty_like(x2)
        hout = torch.empty_like(x2) if res is not None else None
        rstd = _ws(Nr, dev)
        mean = None if rms else _ws(Nr, dev)
        res2 = _c(res).view(-1, H) if res is not None else None  # referenced until the launch
        N.call("pa_norm_fwd", N.dt(x2), int(rms), N.ptr(x2), N.ptr(res2),
               N.ptr(w), N.ptr(b), N.ptr(y), N.ptr(hout), N.ptr(mean), N.ptr(rstd), Nr, H, float(eps), N.stream())
        h = hout if res is not None else x2
        ctx.save_for_backward(h, w, mean, rstd)
        ctx.rms, ctx.has_res, ctx.has_b, ctx.shape = rms, res is not None, b is not None, x.shape
        if res is not None:
            return y.view(x.shape), hout.view(x.shape)
        return y.view(x.shape), None

    @staticmethod
    def backward(ctx, dy, dh):
        h, w, mean, rstd = ctx.saved_tensors
        H = h.shape[-1]
        Nr = h.shape[0]
        dy2 = _c(dy).view(-1, H)
        dres = _c(dh).view(-1, H) if (ctx.has_res and dh is not None) else None
        dx = torch.empty_like(h)
        dw = torch.empty_like(w)
        db = torch.empty_like(w) if ctx.has_b else None
        G = min(1024, (Nr + 3) // 4)  # workspace for the kernel's block cap (norm.hip)
        ws = _ws(2 * max(G, 1) * H, h.device)
        N.call("pa_norm_bwd", N.dt(h), int(ctx.rms), N.ptr(dy2), N.ptr(h), N.ptr(w), N.ptr(mean), N.ptr(rstd),
               N.ptr(dres), N.ptr(dx), N.ptr(dw), N.ptr(db), N.ptr(ws), Nr, H, N.stream())
        dx = dx.view(ctx.shape)
        return dx, (dx if ctx.has_res else None), dw, db, None, None


def layer_norm_stats(x2, w, b, eps):
    """Fluid layer_norm forward on the norm kernel: rows of ``x2`` [N, H] ->
    (y, mean [N] fp32, rstd [N] fp32) -- the statistics come from the same pass."""
    Nr, H = x2.shape
    x2 = _c(x2)
    y = torch.empty_like(x2)
    mean, rstd = _ws(Nr, x2.device), _ws(Nr, x2.device)
    N.call("pa_norm_fwd", N.dt(x2), 0, N.ptr(x2), None, N.ptr(w), N.ptr(b), N.ptr(y), None, N.ptr(mean),
           N.ptr(rstd), Nr, H, float(eps), N.stream())
    return y, mean, rstd


def layer_norm_stats_grad(dy2, x2, w, mean, rstd, has_b):
    """Backward of :func:`layer_norm_stats` from the saved statistics -> (dx, dw, db)."""
    Nr, H = x2.shape
    x2, dy2 = _c(x2), _c(dy2)
    dx = torch.empty_like(x2)
    dw = torch.empty_like(w)
    db = torch.empty_like(w) if has_b else None
    G = min(1024, (Nr + 3) // 4)  # workspace for the kernel's block cap (norm.hip)
    ws = _ws(2 * max(G, 1) * H, x2.device)
    N.call("pa_norm_bwd", N.dt(x2), 0, N.ptr(dy2), N.ptr(x2), N.ptr(w), N.ptr(_c(mean)), N.ptr(_c(rstd)), None,
           N.ptr(dx), N.ptr(dw), N.ptr(db), N.ptr(ws), Nr, H, N.stream())
    return dx, dw, db


def norm_kernel_ok(x2, w):
    return (x2.is_cuda and w is not None and x2.dtype in (torch.float32, torch.bfloat16) and w.dtype == x2.dtype
            and x2.shape[-1] % 8 == 0 and x2.shape[-1] <= 8192 and x2.shape[0] > 0)


def param_ready(w):
    """Wait for a deferred parameter all-gather (``FlatShardedOptimizer`` with
    ``overlap_allgather``) before the first read of ``w`` in a step."""
    f = getattr(w, "_pa_pending", None)
    if f is not None:
        f(w)


class _NormRefFn(torch.autograd.Function):
    """Host / unsupported-shape RMSNorm / LayerNorm (optionally fused residual add)
    with its analytic backward, so the reverse pass stays on the framework tape."""

    @staticmethod
    def forward(ctx, x, res, w, b, eps, rms):
        h = x.float() + res.float() if res is not None else x.float()
        if rms:
            rstd = torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + eps)
            xhat = h * rstd
        else:
            xc = h - h.mean(-1, keepdim=True)
            rstd = torch.rsqrt(xc.pow(2).mean(-1, keepdim=True) + eps)
            xhat = xc * rstd
        y = xhat * w.float()
        if b is not None:
            y = y + b.float()
        ctx.save_for_backward(xhat, rstd, w)
        ctx.meta = (rms, res is not None, b is not None, x.dtype, None if res is None else res.dtype)
        return y.to(x.dtype), (h.to(x.dtype) if res is not None else None)

    @staticmethod
    def backward(ctx, dy, dh):
        xhat, rstd, w = ctx.saved_tensors
        rms, has_res, has_b, xdt, rdt = ctx.meta
        H = xhat.shape[-1]
        dyf = dy.float()
        dw = (dyf * xhat).reshape(-1, H).sum(0).to(w.dtype)
        db = dyf.reshape(-1, H).sum(0).to(w.dtype) if has_b else None
        g = dyf * w.float()
        proj = (g * xhat).mean(-1, keepdim=True)
        dx = rstd * (g - xhat * proj) if rms else rstd * (g - g.mean(-1, keepdim=True) - xhat * proj)
        if has_res and dh is not None:
            dx = dx + dh.float()
        return dx.to(xdt), (dx.to(rdt) if has_res else None), dw, db, None, None


def rms_norm(x, weight, eps=1e-6, residual=None):
    """y = x * rsqrt(mean(x^2) + eps) * weight.  With ``residual``: h = x + residual,
    returns (rms_norm(h), h) with the add fused into the same pass."""
    param_ready(weight)
    if x.is_cuda:
        y, h = _tape.apply(_NormFn, x, residual, weight, None, eps, True)
        return (y, h) if residual is not None else y
    y, h = _tape.apply(_NormRefFn, x, residual, weight, None, eps, True)
    return (y, h) if residual is not None else y


def layer_norm(x, weight, bias=None, eps=1e-5, residual=None):
    if weight is not None:
        param_ready(weight)
    if bias is not None:
        param_ready(bias)
    if x.is_cuda and weight is not None and x.shape[-1] % 8 == 0 and x.shape[-1] <= 8192:
        y, h = _tape.apply(_NormFn, x, residual, weight, bias, eps, False)
        return (y, h) if residual is not None else y
    if weight is None:
        h = x + residual if residual is not None else x
        y = torch.nn.functional.layer_norm(h, h.shape[-1:], None, bias, eps)
        return (y, h) if residual is not None else y
    y, h = _tape.apply(_NormRefFn, x, residual, weight, bias, eps, False)
    return (y, h) if residual is not None else y


# ====================================================================== rotary


def rope_tables(seq_len: int, head_dim: int, base: float = 10000.0, device=None):
    inv = 1.0 / (base ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    t = torch.arange(seq_len, dtype=torch.float64)
    f = torch.outer(t, inv)
    return f.cos().float().contiguous().to(device), f.sin().float().contiguous().to(device)


def _rope_ref(x, cos, sin, sign=1.0):
    # x [..., S, nh, D] (token dim = -3)
    D = x.shape[-1]
    S = x.shape[-3]
    c = cos[:S].view(S, 1, D // 2)
    s = sin[:S].view(S, 1, D // 2) * sign
    a, b = x[..., : D // 2].float(), x[..., D // 2:].float()
    return torch.cat([a * c - b * s, b * c + a * s], -1).to(x.dtype)


# ====================================================================== flash attention


def _attn_ref(q, k, v, causal, scale):
    # [B, S, H, D] layout
    B, Sq, Hq, D = q.shape
    Hk = k.shape[2]
    if Hk != Hq:
        k = k.repeat_interleave(Hq // Hk, dim=2)
        v = v.repeat_interleave(Hq // Hk, dim=2)
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        Sk = k.shape[1]
        m = torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).tril(Sk - Sq)
        s = s.masked_fill(~m, float("-inf"))
    p = torch.softmax(s, -1)
    o = torch.matmul(p, vf).transpose(1, 2)
    return o.to(q.dtype)


def _fa_strides(t):
    # [B, S, H, D] view with unit stride on D
    assert t.stride(-1) == 1, "flash attention needs a unit stride on the head dim"
    return [t.stride(0), t.stride(1), t.stride(2)]


def _fa_fwd(q, k, v, causal, scale, out=None):
    B, Sq, Hq, D = q.shape
    Sk, Hk = k.shape[1], k.shape[2]
    o = torch.empty(B, Sq, Hq, D, dtype=q.dtype, device=q.device) if out is None else out
    lse = torch.empty(B, Hq, Sq, dtype=torch.float32, device=q.device)
    st = ctypes_long_array(_fa_strides(q) + _fa_strides(k) + _fa_strides(v) + _fa_strides(o))
    N.call("pa_flash_attn_fwd", N.ptr(q), N.ptr(k), N.ptr(v), N.ptr(o), N.ptr(lse), st,
           B, Sq, Sk, Hq, Hk, D, float(scale), int(causal), N.stream())
    return o, lse


def _fa_bwd(q, k, v, o, do, lse, causal, scale, dk, dv, dq_rope_out=None):
    """dk/dv: [B, Sk, Hq, D] views (expanded over q heads) written by the kernel.

    Returns the fp32 dQ accumulator [B, Sq, Hq, D] -- or, with ``dq_rope_out =
    (out, row_stride, cos, sin)`` on the partial-slab path, writes the
    inverse-rotated bf16 dQ straight into ``out`` and returns None."""
    B, Sq, Hq, D = q.shape
    Sk, Hk = k.shape[1], k.shape[2]
    delta = torch.empty(B, Hq, Sq, dtype=torch.float32, device=q.device)
    st = ctypes_long_array(_fa_strides(q) + _fa_strides(k) + _fa_strides(v) + _fa_strides(o)
                           + _fa_strides(do) + _fa_strides(dk))
    assert dk.stride() == dv.stride()
    part = None
    kblk = N.lib().pa_fa_bwd_part_kblk(Sq, Sk, D, int(causal))
    nkb = (Sk + kblk - 1) // kblk if kblk else 0
    if kblk:
        # per-key-block dQ partial slabs (plain stores) summed by a reduce kernel
        part = torch.empty(nkb, B, Hq, Sq, D, dtype=torch.bfloat16, device=q.device)
    fused = part is not None and dq_rope_out is not None
    dq_acc = None if fused else torch.empty(B, Sq, Hq, D, dtype=torch.float32, device=q.device)
    N.call("pa_flash_attn_bwd", N.ptr(q), N.ptr(k), N.ptr(v), N.ptr(o), N.ptr(do), N.ptr(lse),
           N.ptr(delta), N.ptr(dq_acc), N.ptr(dk), N.ptr(dv), st, B, Sq, Sk, Hq, Hk, D,
           float(scale), int(causal), N.ptr(part), N.stream())
    if fused:
        out, ts, cos, sin = dq_rope_out
        assert cos.dtype == torch.float32 and cos.is_contiguous() and sin.is_contiguous()
        assert cos.shape[0] >= Sq and cos.shape[1] == D // 2
        N.call("pa_fa_dq_reduce_rope", N.ptr(part), nkb, B, Sq, Sk, Hq, int(causal), N.ptr(out), ts,
               N.ptr(cos), N.ptr(sin), kblk, N.stream())
    return dq_acc


_FA_SPLIT = os.environ.get("FLAGS_fa_bwd_split", "1") not in ("0", "false", "False")


def _fa_bwd_split(q, k, v, o, do, lse, causal, scale, dq, dk, dv, cos=None, sin=None):
    """The two-kernel flash-attention backward (csrc/kernels/fa_bwd_split.hip): dQ
    (query-stationary, computes delta itself) then dK / dV (key-stationary, GQA group
    summed in registers), bf16 results written straight into ``dq`` [B, Sq, Hq, D] and
    ``dk`` / ``dv`` [B, Sk, Hkv, D] (any strides with unit D stride), with the inverse
    rotary applied to dq / dk when ``cos`` / ``sin`` are given.  Returns False (nothing
    written) when the shape is not covered (D != 128, 32-bit offsets)."""
    if not _FA_SPLIT:
        return False
    B, Sq, Hq, D = q.shape
    Sk, Hk = k.shape[1], k.shape[2]
    st = ctypes_long_array(_fa_strides(q) + _fa_strides(k) + _fa_strides(v) + _fa_strides(o) + _fa_strides(do)
                           + _fa_strides(dq) + _fa_strides(dk) + _fa_strides(dv))
    if not N.lib().pa_fa_bwd_split_ok(B, Sq, Sk, Hq, Hk, D, st):
        return False
    if cos is not None:
        assert cos.dtype == torch.float32 and cos.is_contiguous() and sin.is_contiguous()
        assert cos.shape[0] >= max(Sq, Sk) and cos.shape[1] == D // 2
    ld2 = torch.empty(B, Hq, Sq, 2, dtype=torch.float32, device=q.device)
    N.call("pa_fa_bwd_split", N.ptr(q), N.ptr(k), N.ptr(v), N.ptr(o), N.ptr(do), N.ptr(lse), N.ptr(ld2),
           N.ptr(dq), N.ptr(dk), N.ptr(dv), st, B, Sq, Sk, Hq, Hk, D, float(scale), int(causal),
           N.ptr(cos), N.ptr(sin), N.stream())
    return True


def ctypes_long_array(vals):
    import ctypes
    return (ctypes.c_long * len(vals))(*[int(x) for x in vals])


class _FlashAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        o, lse = _fa_fwd(q, k, v, causal, scale)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        do = _c(do)
        B, Sq, Hq, D = q.shape
        Sk, Hk = k.shape[1], k.shape[2]
        dq = torch.empty_like(q)
        dkk, dvv = torch.empty_like(k), torch.empty_like(v)
        if _fa_bwd_split(q, k, v, o, do, lse, ctx.causal, ctx.scale, dq, dkk, dvv):
            return dq, dkk, dvv, None, None
        dk = torch.empty(B, Sk, Hq, D, dtype=q.dtype, device=q.device)
        dv = torch.empty_like(dk)
        dq_acc = _fa_bwd(q, k, v, o, do, lse, ctx.causal, ctx.scale, dk, dv)
        dq = dq_acc.to(q.dtype)
        if Hk != Hq:
            dk = dk.view(B, Sk, Hk, Hq // Hk, D).sum(3)
            dv = dv.view(B, Sk, Hk, Hq // Hk, D).sum(3)
        return dq, dk, dv, None, None


def flash_attention(q, k, v, causal=True, scale=None):
    """Fused attention over [B, S, H, D] tensors (GQA when k/v have fewer heads).
    Head dims 64 / 128 run the tuned kernels; 256 runs the same kernels
    instantiated at D = 256 (register-spilling: a correctness path)."""
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    if q.is_cuda:
        if q.dtype != torch.bfloat16 or q.shape[-1] not in (64, 128, 256):
            raise NotImplementedError("flash_attention kernel: bf16 with head_dim 64/128/256")
        return _tape.apply(_FlashAttnFn, q, k, v, causal, scale)
    return _attn_ref(q, k, v, causal, scale)


class _FlashAttnVarlenFn(torch.autograd.Function):
    """Packed variable-length batch: sequence i owns rows [cu_q[i], cu_q[i+1]) of q and
    [cu_k[i], cu_k[i+1]) of k / v.  Each sequence runs the flash kernels on strided
    [1, L, H, D] views of the packed tensors (no padding, no copies in, the output
    written in place); the per-sequence launches are the varlen schedule."""

    @staticmethod
    def forward(ctx, q, k, v, cu_q, cu_k, causal, scale):
        o = torch.empty_like(q)
        lses = []
        for i in range(len(cu_q) - 1):
            a, b, c, d = cu_q[i], cu_q[i + 1], cu_k[i], cu_k[i + 1]
            if b == a:
                lses.append(None)
                continue
            if d == c:
                o[a:b].zero_()
                lses.append(None)
                continue
            _, lse = _fa_fwd(q[a:b].unsqueeze(0), k[c:d].unsqueeze(0), v[c:d].unsqueeze(0), causal, scale,
                             out=o[a:b].unsqueeze(0))
            lses.append(lse)
        ctx.save_for_backward(q, k, v, o)
        ctx.lses, ctx.cu_q, ctx.cu_k, ctx.causal, ctx.scale = lses, cu_q, cu_k, causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o = ctx.saved_tensors
        do = _c(do)
        Hq, Hk, D = q.shape[1], k.shape[1], q.shape[2]
        dq = torch.zeros_like(q)
        dk = torch.zeros(k.shape[0], Hq, D, dtype=q.dtype, device=q.device)
        dv = torch.zeros_like(dk)
        for i, lse in enumerate(ctx.lses):
            if lse is None:
                continue
            a, b, c, d = ctx.cu_q[i], ctx.cu_q[i + 1], ctx.cu_k[i], ctx.cu_k[i + 1]
            acc = _fa_bwd(q[a:b].unsqueeze(0), k[c:d].unsqueeze(0), v[c:d].unsqueeze(0), o[a:b].unsqueeze(0),
                          do[a:b].unsqueeze(0), lse, ctx.causal, ctx.scale, dk[c:d].unsqueeze(0),
                          dv[c:d].unsqueeze(0))
            dq[a:b] = acc[0].to(q.dtype)
        if Hk != Hq:
            dk = dk.view(-1, Hk, Hq // Hk, D).sum(2)
            dv = dv.view(-1, Hk, Hq // Hk, D).sum(2)
        return dq, dk, dv, None, None, None, None


def flash_attention_varlen(q, k, v, cu_seqlens_q, cu_seqlens_k=None, causal=True, scale=None):
    """Attention over packed variable-length sequences: q [total_q, Hq, D], k / v
    [total_k, Hk, D], cu_seqlens_* host lists (or tensors) of n+1 offsets (the LoD
    of the reference's sequence ops).  Returns [total_q, Hq, D]."""
    cu_q = [int(x) for x in (cu_seqlens_q.tolist() if torch.is_tensor(cu_seqlens_q) else cu_seqlens_q)]
    cu_k = cu_q if cu_seqlens_k is None else \
        [int(x) for x in (cu_seqlens_k.tolist() if torch.is_tensor(cu_seqlens_k) else cu_seqlens_k)]
    if len(cu_q) != len(cu_k):
        raise ValueError("cu_seqlens_q and cu_seqlens_k describe different batch sizes")
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    if q.is_cuda and q.dtype == torch.bfloat16 and q.shape[-1] in (64, 128, 256):
        return _tape.apply(_FlashAttnVarlenFn, q, k, v, cu_q, cu_k, causal, scale)
    outs = []
    for i in range(len(cu_q) - 1):
        qs, ks, vs = (t[a:b].unsqueeze(0) for t, a, b in ((q, cu_q[i], cu_q[i + 1]), (k, cu_k[i], cu_k[i + 1]),
                                                         (v, cu_k[i], cu_k[i + 1])))
        outs.append(_attn_ref(qs, ks, vs, causal, scale)[0] if ks.shape[1] else torch.zeros_like(qs[0]))
    return torch.cat(outs, 0) if outs else q.new_zeros(q.shape)


class _RopeAttnFn(torch.autograd.Function):
    """Fused rotary + flash attention over a packed QKV projection output.

    qkv: [B, S, (Hq + 2*Hk) * D].  Forward repacks rotated q|k plus v into one
    buffer in a single pass (the only activation saved), runs the attention
    kernel on strided views of it; backward writes dk/dv straight into the
    packed dqkv gradient and fuses the fp32 dq-accumulator cast with the inverse
    rotation, so dqkv feeds the QKV GEMM backward with no copies.
    """

    @staticmethod
    def forward(ctx, qkv, cos, sin, Hq, Hk, D, causal, scale):
        B, S, W = qkv.shape
        nh = Hq + 2 * Hk
        qkv = _c(qkv)
        packed = torch.empty_like(qkv)
        N.call("pa_rope", 1, 1, N.ptr(qkv), W, N.ptr(packed), W, N.ptr(cos), N.ptr(sin), None,
               B, S, nh, Hq + Hk, D, 0, N.stream())
        p4 = packed.view(B, S, nh, D)
        q, k, v = p4[:, :, :Hq], p4[:, :, Hq:Hq + Hk], p4[:, :, Hq + Hk:]
        o, lse = _fa_fwd(q, k, v, causal, scale)
        ctx.save_for_backward(packed, o, lse, cos, sin)
        ctx.cfg = (Hq, Hk, D, causal, scale)
        return o.view(B, S, Hq * D)

    @staticmethod
    def backward(ctx, do):
        packed, o, lse, cos, sin = ctx.saved_tensors
        Hq, Hk, D, causal, scale = ctx.cfg
        return (_rope_attn_backward(packed, o, lse, cos, sin, do, Hq, Hk, D, causal, scale),
                None, None, None, None, None, None, None)


def _rope_attn_backward(packed, o, lse, cos, sin, do, Hq, Hk, D, causal, scale):
    """dqkv [B, S, (Hq+2Hk)*D] (un-rotated projection gradient) of rotary + flash
    attention, from the packed rotated q|k|v the forward saved."""
    B, S, W = packed.shape
    nh = Hq + 2 * Hk
    p4 = packed.view(B, S, nh, D)
    q, k, v = p4[:, :, :Hq], p4[:, :, Hq:Hq + Hk], p4[:, :, Hq + Hk:]
    do = _c(do).view(B, S, Hq, D)
    dqkv = torch.empty_like(packed)
    d4 = dqkv.view(B, S, nh, D)
    # two-kernel backward: dq / dk inverse-rotated, GQA-summed and stored in bf16 straight
    # into dqkv's slots -- no dQ slabs, no reduce, no dk rotary pass, no GQA fold
    if _fa_bwd_split(q, k, v, o, do, lse, causal, scale, d4[:, :, :Hq], d4[:, :, Hq:Hq + Hk],
                     d4[:, :, Hq + Hk:], cos, sin):
        return dqkv
    # dq: summed, inverse-rotated and cast straight into dqkv's dq slot when the
    # partial-slab kernel runs (else via the fp32 accumulator + one rope pass)
    rope_out = (dqkv, W, cos, sin)
    if Hk == Hq:
        dk, dv = d4[:, :, Hq:2 * Hq], d4[:, :, 2 * Hq:]
        dq_acc = _fa_bwd(q, k, v, o, do, lse, causal, scale, dk, dv, rope_out)
    else:
        dk_e = torch.empty(B, S, Hq, D, dtype=packed.dtype, device=packed.device)
        dv_e = torch.empty_like(dk_e)
        dq_acc = _fa_bwd(q, k, v, o, do, lse, causal, scale, dk_e, dv_e, rope_out)
        # fold the per-query-head dK / dV over each kv head's group straight into
        # dqkv's k / v slots (one fp32-summing pass)
        N.call("pa_fa_gqa_fold", N.ptr(dk_e), N.ptr(dv_e), N.ptr(d4[:, :, Hq:Hq + Hk]),
               N.ptr(d4[:, :, Hq + Hk:]), B * S, Hq, Hk, D, nh * D, N.stream())
    if dq_acc is not None:
        N.call("pa_rope", 0, 1, N.ptr(dq_acc), Hq * D, N.ptr(dqkv), W, N.ptr(cos), N.ptr(sin), None,
               B, S, Hq, Hq, D, 1, N.stream())
    # dk: inverse rotation in place inside dqkv
    kview = dqkv.view(B, S, nh * D)[:, :, Hq * D:]
    N.call("pa_rope", 1, 1, N.ptr(kview), W, N.ptr(kview), W, N.ptr(cos), N.ptr(sin), None,
           B, S, Hk, Hk, D, 1, N.stream())
    return dqkv


class _QKVRopeAttnFn(torch.autograd.Function):
    """The QKV projection, rotary embedding and flash attention as one node.

    Forward: one GEMM whose epilogue applies the neox rotation to the q / k columns
    (``gemm_epi(EPI_ROPE)``), writing the packed rotated q|k|v the attention kernel
    reads -- the projection output is never re-read by a separate rotary pass.
    Backward: the attention backward produces the un-rotated dqkv (as
    ``_RopeAttnFn``), then the projection's dX / dW GEMMs (as ``_LinearFn``)."""

    @staticmethod
    def forward(ctx, y, w, cos, sin, Hq, Hk, D, causal, scale):
        K, W = w.shape
        y2 = y.reshape(-1, K)
        T = y2.shape[0]
        S = y.shape[-2]
        wt = _weight_t(w, T)
        packed = torch.empty(T, W, dtype=y.dtype, device=y.device)
        _G.gemm_epi(_G.EPI_ROPE, _c(y2), wt, T, W, K, out=packed, cos=cos, sin=sin, rope_cols=(Hq + Hk) * D,
                    rope_S=S)
        packed = packed.view(*y.shape[:-1], W)
        B = packed.shape[0]
        p4 = packed.view(B, S, Hq + 2 * Hk, D)
        o, lse = _fa_fwd(p4[:, :, :Hq], p4[:, :, Hq:Hq + Hk], p4[:, :, Hq + Hk:], causal, scale)
        ctx.save_for_backward(y, w, packed, o, lse, cos, sin)
        ctx.cfg = (Hq, Hk, D, causal, scale)
        return o.view(B, S, Hq * D)

    @staticmethod
    def backward(ctx, do):
        y, w, packed, o, lse, cos, sin = ctx.saved_tensors
        Hq, Hk, D, causal, scale = ctx.cfg
        dqkv = _rope_attn_backward(packed, o, lse, cos, sin, do, Hq, Hk, D, causal, scale)
        dx, dw = _linear_bwd(ctx, y, w, dqkv, ctx.needs_input_grad[0], ctx.needs_input_grad[1])
        return dx, dw, None, None, None, None, None, None, None


def _qkv_rope_fused_ok(y, w, cos, Hq, Hk):
    K, W = w.shape
    T = y.numel() // K
    D = W // (Hq + 2 * Hk)
    return (y.is_cuda and y.dtype == torch.bfloat16 and D == 128 and y.dim() == 3 and K % 64 == 0
            and cos.dtype == torch.float32 and cos.is_contiguous() and cos.shape[-1] == 64
            and _G.epi_supported(T, W, K, y.reshape(-1, K), w) and _weight_t(w, T) is not None)


def qkv_rope_attention(y, w_qkv, cos, sin, num_heads, num_kv_heads=None, causal=True, scale=None):
    """rope_attention(linear(y, w_qkv), ...) with the rotary fused into the projection
    GEMM's epilogue on the GPU (D = 128); the unfused ops elsewhere."""
    Hk = num_kv_heads or num_heads
    param_ready(w_qkv)
    D = w_qkv.shape[1] // (num_heads + 2 * Hk)
    if scale is None:
        scale = 1.0 / math.sqrt(D)
    if _qkv_rope_fused_ok(y, w_qkv, cos, num_heads, Hk):
        return _tape.apply(_QKVRopeAttnFn, y, w_qkv, cos, sin, num_heads, Hk, D, causal, scale)
    return rope_attention(linear(y, w_qkv), cos, sin, num_heads, Hk, causal=causal, scale=scale)


class _PackedAttnRefFn(torch.autograd.Function):
    """Host / unsupported-shape attention over a packed [B, S, (Hq+2Hk)*D] projection,
    with the neox rotary on q / k when ``cos`` is given, and its analytic backward
    (dV = P^T dO, dS = P (dO V^T - rowsum(dO O)), dQ = s dS K, dK = s dS^T Q; the
    rotary's backward is the inverse rotation; GQA gradients summed per kv head)."""

    @staticmethod
    def forward(ctx, qkv, cos, sin, Hq, Hk, D, causal, scale):
        B, S, W = qkv.shape
        x = qkv.float().view(B, S, Hq + 2 * Hk, D)
        q, k, v = x[:, :, :Hq], x[:, :, Hq:Hq + Hk], x[:, :, Hq + Hk:]
        if cos is not None:
            q, k = _rope_ref(q, cos, sin), _rope_ref(k, cos, sin)
        r = Hq // Hk
        ke, ve = k.repeat_interleave(r, 2), v.repeat_interleave(r, 2)
        s_ = torch.einsum("bqhd,bkhd->bhqk", q, ke) * scale
        if causal:
            s_ = s_.masked_fill(torch.ones(S, S, dtype=torch.bool, device=s_.device).triu(1), float("-inf"))
        p_ = torch.softmax(s_, -1)
        o = torch.einsum("bhqk,bkhd->bqhd", p_, ve)
        ctx.save_for_backward(q, ke, ve, p_, o, cos, sin)
        ctx.meta = (Hq, Hk, D, scale, qkv.dtype)
        return o.reshape(B, S, Hq * D).to(qkv.dtype)

    @staticmethod
    def backward(ctx, do):
        q, ke, ve, p_, o, cos, sin = ctx.saved_tensors
        Hq, Hk, D, scale, dt = ctx.meta
        B, S = q.shape[:2]
        do = do.float().view(B, S, Hq, D)
        dv = torch.einsum("bhqk,bqhd->bkhd", p_, do)
        dp = torch.einsum("bqhd,bkhd->bhqk", do, ve)
        delta = (do * o).sum(-1).permute(0, 2, 1).unsqueeze(-1)
        ds = p_ * (dp - delta) * scale
        dq = torch.einsum("bhqk,bkhd->bqhd", ds, ke)
        dk = torch.einsum("bhqk,bqhd->bkhd", ds, q)
        r = Hq // Hk
        dk = dk.view(B, S, Hk, r, D).sum(3)
        dv = dv.view(B, S, Hk, r, D).sum(3)
        if cos is not None:
            dq, dk = _rope_ref(dq, cos, sin, sign=-1.0), _rope_ref(dk, cos, sin, sign=-1.0)
        dqkv = torch.cat([dq, dk, dv], 2).reshape(B, S, (Hq + 2 * Hk) * D)
        return dqkv.to(dt), None, None, None, None, None, None, None


def rope_attention(qkv, cos, sin, num_heads, num_kv_heads=None, causal=True, scale=None):
    """Rotary (neox) + causal flash attention on a packed [B, S, (Hq+2Hk)*D] tensor.
    Returns [B, S, Hq*D]."""
    Hk = num_kv_heads or num_heads
    B, S, W = qkv.shape
    D = W // (num_heads + 2 * Hk)
    if scale is None:
        scale = 1.0 / math.sqrt(D)
    if qkv.is_cuda and qkv.dtype == torch.bfloat16 and D in (64, 128):
        return _tape.apply(_RopeAttnFn, qkv, cos, sin, num_heads, Hk, D, causal, scale)
    # other dtypes / head sizes: plain rotary + attention (the kernels are bf16)
    return _tape.apply(_PackedAttnRefFn, qkv, cos[:S], sin[:S], num_heads, Hk, D, causal, scale)


_IDENT_ROPE = {}


def _identity_rope(S, D, device):
    """cos = 1, sin = 0 tables: lets the no-rotary path reuse the fused dQ
    slab-reduce + bf16 store into the packed gradient (``pa_fa_dq_reduce_rope``)."""
    key = (S, D, str(device))
    t = _IDENT_ROPE.get(key)
    if t is None:
        t = (_fill_native(torch.empty(S, D // 2, dtype=torch.float32, device=device), 1.0),
             _fill_native(torch.empty(S, D // 2, dtype=torch.float32, device=device), 0.0))
        _IDENT_ROPE[key] = t
    return t


class _PackedAttnFn(torch.autograd.Function):
    """Causal flash attention straight off a packed [B, S, 3*H*D] QKV projection
    (GPT / ERNIE layout q|k|v): the kernel reads strided q/k/v views of the GEMM
    output (no split copies), backward writes dq/dk/dv into one packed dqkv --
    instead of autograd's three zero-filled select-backward buffers and two adds."""

    @staticmethod
    def forward(ctx, qkv, H, D, causal, scale):
        B, S, W = qkv.shape
        qkv = _c(qkv)
        p4 = qkv.view(B, S, 3 * H, D)
        o, lse = _fa_fwd(p4[:, :, :H], p4[:, :, H:2 * H], p4[:, :, 2 * H:], causal, scale)
        ctx.save_for_backward(qkv, o, lse)
        ctx.cfg = (H, D, causal, scale)
        return o.view(B, S, H * D)

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        H, D, causal, scale = ctx.cfg
        B, S, W = qkv.shape
        p4 = qkv.view(B, S, 3 * H, D)
        do = _c(do).view(B, S, H, D)
        dqkv = torch.empty_like(qkv)
        d4 = dqkv.view(B, S, 3 * H, D)
        if _fa_bwd_split(p4[:, :, :H], p4[:, :, H:2 * H], p4[:, :, 2 * H:], o, do, lse, causal, scale,
                         d4[:, :, :H], d4[:, :, H:2 * H], d4[:, :, 2 * H:]):
            return dqkv, None, None, None, None
        cos, sin = _identity_rope(S, D, qkv.device)
        dq_acc = _fa_bwd(p4[:, :, :H], p4[:, :, H:2 * H], p4[:, :, 2 * H:], o, do, lse, causal, scale,
                         d4[:, :, H:2 * H], d4[:, :, 2 * H:], (dqkv, W, cos, sin))
        if dq_acc is not None:
            N.call("pa_rope", 0, 1, N.ptr(dq_acc), H * D, N.ptr(dqkv), W, N.ptr(cos), N.ptr(sin), None,
                   B, S, H, H, D, 1, N.stream())
        return dqkv, None, None, None, None


def packed_attention(qkv, num_heads, causal=True, scale=None):
    """Flash attention on a packed [B, S, 3*H*D] (q|k|v) tensor; returns [B, S, H*D]."""
    B, S, W = qkv.shape
    D = W // (3 * num_heads)
    if scale is None:
        scale = 1.0 / math.sqrt(D)
    if qkv.is_cuda and qkv.dtype == torch.bfloat16 and D in (64, 128):
        return _tape.apply(_PackedAttnFn, qkv, num_heads, D, causal, scale)
    return _tape.apply(_PackedAttnRefFn, qkv, None, None, num_heads, num_heads, D, causal, scale)


def apply_rotary(x, cos, sin, inverse=False):
    """Rotate [B, S, H, D] (neox convention)."""
    if x.is_cuda:
        return _tape.apply(_RopeFn, x, cos, sin, inverse)
    return _rope_ref(x, cos, sin, -1.0 if inverse else 1.0)


class _RopeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cos, sin, inverse):
        x = _c(x)
        B, S, H, D = x.shape
        y = torch.empty_like(x)
        N.call("pa_rope", N.dt(x), N.dt(y), N.ptr(x), H * D, N.ptr(y), H * D, N.ptr(cos), N.ptr(sin), None,
               B, S, H, H, D, int(inverse), N.stream())
        ctx.save_for_backward(cos, sin)
        ctx.inverse = inverse
        return y

    @staticmethod
    def backward(ctx, dy):
        cos, sin = ctx.saved_tensors
        dy = _c(dy)
        B, S, H, D = dy.shape
        dx = torch.empty_like(dy)
        N.call("pa_rope", N.dt(dy), N.dt(dx), N.ptr(dy), H * D, N.ptr(dx), H * D, N.ptr(cos), N.ptr(sin), None,
               B, S, H, H, D, int(not ctx.inverse), N.stream())
        return dx, None, None, None


# ====================================================================== SwiGLU


class _SwiGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu):
        gu = _c(gu)
        I2 = gu.shape[-1]
        I = I2 // 2
        Nr = gu.numel() // I2
        out = torch.empty(*gu.shape[:-1], I, dtype=gu.dtype, device=gu.device)
        N.call("pa_swiglu_fwd", N.dt(gu), N.ptr(gu), N.ptr(out), Nr, I, N.stream())
        ctx.save_for_backward(gu)
        return out

    @staticmethod
    def backward(ctx, dout):
        (gu,) = ctx.saved_tensors
        dout = _c(dout)
        I2 = gu.shape[-1]
        dgu = torch.empty_like(gu)
        N.call("pa_swiglu_bwd", N.dt(gu), N.ptr(gu), N.ptr(dout), N.ptr(dgu), gu.numel() // I2, I2 // 2, N.stream())
        return dgu


def swiglu(x, y=None):
    """silu(gate) * up.  With one argument, x = [gate | up] along the last axis."""
    if y is not None:
        x = torch.cat([x, y], -1)
    if x.is_cuda and (x.shape[-1] // 2) % 8 == 0:
        return _tape.apply(_SwiGLUFn, x)
    return _tape.apply(_SwiGLURefFn, x)


class _SwiGLURefFn(torch.autograd.Function):
    """Host SwiGLU over [gate | up] with its analytic backward."""

    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        g, u = x.float().chunk(2, -1)
        return (torch.nn.functional.silu(g) * u).to(x.dtype)

    @staticmethod
    def backward(ctx, d):
        (x,) = ctx.saved_tensors
        g, u = x.float().chunk(2, -1)
        sg = torch.sigmoid(g)
        d = d.float()
        return torch.cat([d * u * sg * (1 + g * (1 - sg)), d * g * sg], -1).to(x.dtype)


# ---------------------------------------------------------------- fused SwiGLU MLP
# gate|up projections stored interleaved in blocks of SWIGLU_BLOCK columns (block b:
# gate columns 32b..32b+15, up columns 32b+16..32b+31), so one GEMM tile holds both
# halves of every SwiGLU input and the activation runs in the projection's epilogue.
SWIGLU_BLOCK = 16


def deinterleave_gate_up(gu, block=SWIGLU_BLOCK):
    """[..., 2I] interleaved gate|up -> (gate [..., I], up [..., I])."""
    *lead, n2 = gu.shape
    v = gu.reshape(*lead, n2 // (2 * block), 2, block)
    return v[..., 0, :].reshape(*lead, n2 // 2), v[..., 1, :].reshape(*lead, n2 // 2)


def interleave_gate_up(g, u, block=SWIGLU_BLOCK):
    """(gate [..., I], up [..., I]) -> [..., 2I] in the interleaved layout."""
    *lead, n = g.shape
    return torch.stack([g.reshape(*lead, n // block, block), u.reshape(*lead, n // block, block)], -2) \
        .reshape(*lead, 2 * n)


def swiglu_mlp_fused_ok(x, w_gu, w_down):
    K, N2 = w_gu.shape
    T = x.numel() // max(K, 1)
    return (x.is_cuda and x.dtype == torch.bfloat16 and N2 % 32 == 0 and K % 64 == 0 and w_down.shape[1] % 64 == 0
            and _G.epi_supported(T, N2, K, x.reshape(-1, K), w_gu) and _weight_t(w_gu, T) is not None
            and _G.epi_supported(T, N2 // 2, w_down.shape[1], x.reshape(-1, K), w_down))


class _SwiGLUMLPFn(torch.autograd.Function):
    """y = (silu(gate) * up) @ W_down with [gate|up] = x @ W_gu (interleaved layout).

    GPU: the gate|up GEMM writes gu (kept for the backward) AND h = silu(gate) * up
    from its epilogue (``EPI_SWIGLU_FWD``); the backward's da = dY W_down^T GEMM turns
    into d(gate|up) in its epilogue (``EPI_SWIGLU_BWD``), so neither h's input pass nor
    da ever reach memory; then the usual dW / dX GEMMs.  CPU / unsupported shapes:
    the same math with torch ops."""

    @staticmethod
    def forward(ctx, x, w_gu, w_down):
        K, N2 = w_gu.shape
        x2 = x.reshape(-1, K)
        T = x2.shape[0]
        fused = swiglu_mlp_fused_ok(x, w_gu, w_down)
        if fused:
            gu = torch.empty(T, N2, dtype=x.dtype, device=x.device)
            h = torch.empty(T, N2 // 2, dtype=x.dtype, device=x.device)
            _G.gemm_epi(_G.EPI_SWIGLU_FWD, _c(x2), _weight_t(w_gu, T), T, N2, K, out=gu, aux=h)
        else:
            gu = _linear_fwd(x2, w_gu, None)
            g, u = deinterleave_gate_up(gu)
            h = (torch.nn.functional.silu(g.float()) * u.float()).to(x.dtype)
        y = _linear_fwd(h, w_down, None)
        ctx.save_for_backward(x, w_gu, w_down, gu, h)
        ctx.fused = fused
        return y.view(*x.shape[:-1], w_down.shape[1])

    @staticmethod
    def backward(ctx, dy):
        x, w_gu, w_down, gu, h = ctx.saved_tensors
        Hd = w_down.shape[1]
        dy2 = _c(dy).reshape(-1, Hd)
        T, I = h.shape
        if ctx.fused:
            dgu = torch.empty(T, 2 * I, dtype=gu.dtype, device=gu.device)
            _G.gemm_epi(_G.EPI_SWIGLU_BWD, dy2, w_down, T, I, Hd, out=dgu, aux=gu)
        else:
            da = (dy2.float() @ w_down.float().t())
            g, u = deinterleave_gate_up(gu.float())
            sg = torch.sigmoid(g)
            dg = da * u * sg * (1 + g * (1 - sg))
            du = da * g * sg
            dgu = interleave_gate_up(dg, du).to(gu.dtype)
        _, dw_down = _linear_bwd(ctx, h, w_down, dy2, False, ctx.needs_input_grad[2])
        dx, dw_gu = _linear_bwd(ctx, x.reshape(-1, x.shape[-1]), w_gu, dgu, ctx.needs_input_grad[0],
                                ctx.needs_input_grad[1])
        return (dx.view(x.shape) if dx is not None else None), dw_gu, dw_down


def swiglu_mlp(x, w_gate_up, w_down):
    """down(silu(gate) * up) with gate|up = x @ w_gate_up stored INTERLEAVED in
    16-column blocks (:func:`interleave_gate_up`) -- one fused node."""
    param_ready(w_gate_up)
    param_ready(w_down)
    return _tape.apply(_SwiGLUMLPFn, x, w_gate_up, w_down)


# ---------------------------------------------------------------- small tape ops
# Elementwise glue that models apply to activations between fused ops (a bias added
# after a row-parallel all-reduce, position embeddings, loss scaling / averaging):
# each is one recorded node with its hand-written backward, so a forward recorded on
# the framework tape never leaves it (torch autograd stays off).


def _sum_to(g, shape):
    """Reduce a broadcast gradient back to ``shape``."""
    if tuple(g.shape) == tuple(shape):
        return g
    lead = g.dim() - len(shape)
    dims = list(range(lead)) + [lead + i for i, n in enumerate(shape) if n == 1 and g.shape[lead + i] != 1]
    return g.sum(dims, keepdim=False).reshape(shape) if dims else g.reshape(shape)


class _AddFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        ctx.shapes = (a.shape, b.shape, a.dtype, b.dtype)
        if a.is_cuda and a.shape == b.shape and a.dtype == b.dtype and a.is_contiguous() and b.is_contiguous():
            from . import oplib

            r = oplib.binary("add", a, b)
            if r is not None:
                return r
        return a + b

    @staticmethod
    def backward(ctx, g):
        sa, sb, da, db = ctx.shapes
        return _sum_to(g, sa).to(da), _sum_to(g, sb).to(db)


def add(a, b):
    """a + b (b broadcast onto a, e.g. a bias) as one recorded node."""
    return _tape.apply(_AddFn, a, b)


class _ScaleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, s):
        ctx.s = s
        return x * s

    @staticmethod
    def backward(ctx, g):
        return _scale_native(g, ctx.s), None


def scale(x, s):
    """x * s for a Python scalar s (loss / accumulate_steps) as one recorded node."""
    return _tape.apply(_ScaleFn, x, float(s))


class _PositionAddFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, table):
        S = x.shape[-2]
        ctx.S, ctx.tshape, ctx.tdtype = S, table.shape, table.dtype
        return x + table[:S].to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        S, H = ctx.S, g.shape[-1]
        if g.is_cuda and g.dtype == ctx.tdtype and _fast_bias_ok(g) and S * H < 2 ** 31:
            # the table gradient is the column sum of g viewed as [B, S * H]: the bias
            # reduction kernel (fp32 partials), rows past S zero-filled
            g2 = _c(g)
            B = g2.numel() // (S * H)
            dt = torch.empty(ctx.tshape, dtype=g.dtype, device=g.device)
            if S < ctx.tshape[0]:
                _fill_native(dt[S:], 0.0)
            part = _ws(int(N.lib().pa_bias_grad_blocks(B, S * H)) * S * H, g.device)
            N.call("pa_bias_act_bwd", N.dt(g2), 0, N.ptr(g2), None, None, N.ptr(dt), N.ptr(part), B, S * H,
                   N.stream())
            return g, dt
        dt = torch.zeros(ctx.tshape, dtype=torch.float32, device=g.device)
        dt[:S] = g.float().reshape(-1, S, H).sum(0)
        return g, dt.to(ctx.tdtype)


def position_add(x, table):
    """x [B, S, H] + table[:S] (learned absolute position embeddings)."""
    return _tape.apply(_PositionAddFn, x, table)


class _MeanValidFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, loss, label, ignore_index):
        valid = (label != ignore_index)
        n = valid.sum().clamp_min(1).to(torch.float32)
        ctx.save_for_backward(valid, n)
        return (loss.float() * valid).sum() / n

    @staticmethod
    def backward(ctx, g):
        valid, n = ctx.saved_tensors
        return (g / n) * valid.to(torch.float32), None, None


def mean_valid(loss, label, ignore_index=-100):
    """Mean of per-token losses over the labels that are not ``ignore_index``."""
    return _tape.apply(_MeanValidFn, loss, label, ignore_index)


class _ReshapeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, shape):
        ctx.shape = x.shape
        return x.reshape(shape)

    @staticmethod
    def backward(ctx, g):
        return g.reshape(ctx.shape), None


def reshape(x, shape):
    """x.reshape(shape) as a recorded node (a plain view of a tape activation would be
    invisible to the tape)."""
    return _tape.apply(_ReshapeFn, x, tuple(shape))


class _RowGatherFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, idx):
        ctx.save_for_backward(idx)
        ctx.rows = x.shape[0]
        return x.index_select(0, idx)

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        dx = torch.zeros((ctx.rows,) + tuple(g.shape[1:]), dtype=g.dtype, device=g.device)
        return dx.index_add_(0, idx, g), None


def row_gather(x, idx):
    """x[idx] along rows (a permutation / selection) as a recorded node."""
    return _tape.apply(_RowGatherFn, x, idx)


class _ConcatRowsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, *xs):
        ctx.sizes = [x.shape[0] for x in xs]
        return torch.cat(xs, 0)

    @staticmethod
    def backward(ctx, g):
        return tuple(g.split(ctx.sizes, 0))


def concat_rows(xs):
    """torch.cat(xs, 0) as a recorded node."""
    return _tape.apply(_ConcatRowsFn, *xs)


class _StackMeanFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, *ts):
        ctx.n = len(ts)
        return torch.stack([t.float() for t in ts]).mean(0)

    @staticmethod
    def backward(ctx, g):
        gi = _scale_native(g, 1.0 / ctx.n)
        return tuple(gi for _ in range(ctx.n))


def stack_mean(ts):
    """Mean of same-shaped tensors (e.g. per-layer MoE balance losses)."""
    return _tape.apply(_StackMeanFn, *ts)


class _CrossEntropyRefFn(torch.autograd.Function):
    """Per-token log-softmax + NLL (fp32) for host / unsupported tensors."""

    @staticmethod
    def forward(ctx, logits, label, ignore_index):
        lf = logits.float().reshape(-1, logits.shape[-1])
        lab = label.reshape(-1).long()
        lse = torch.logsumexp(lf, -1)
        safe = lab.clamp_min(0)
        loss = lse - lf.gather(1, safe.unsqueeze(1)).squeeze(1)
        loss = torch.where(lab == ignore_index, torch.zeros_like(loss), loss)
        ctx.save_for_backward(lf, lab, lse)
        ctx.meta = (logits.shape, logits.dtype, ignore_index)
        return loss.view(label.shape)

    @staticmethod
    def backward(ctx, g):
        lf, lab, lse = ctx.saved_tensors
        shape, dt, ign = ctx.meta
        p = torch.exp(lf - lse.unsqueeze(1))
        p[torch.arange(lab.numel()), lab.clamp_min(0)] -= 1.0
        p = p * (g.reshape(-1, 1).float() * (lab != ign).unsqueeze(1))
        return p.view(shape).to(dt), None, None


def cross_entropy_tokens(logits, label, ignore_index=-100):
    """Per-token cross entropy (fp32) as one recorded node (the host path of
    :func:`softmax_cross_entropy`)."""
    return _tape.apply(_CrossEntropyRefFn, logits, label, ignore_index)


# ====================================================================== softmax CE


class _SoftmaxCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, label, ignore_index, inplace_grad):
        V = logits.shape[-1]
        x = _c(logits).view(-1, V)
        lab = _c(label).view(-1).long()
        Nr = x.shape[0]
        loss = torch.empty(Nr, dtype=torch.float32, device=x.device)
        lse = torch.empty(Nr, dtype=torch.float32, device=x.device)
        N.call("pa_softmax_ce_fwd", N.dt(x), N.ptr(x), N.ptr(lab), None, N.ptr(loss), N.ptr(lse), Nr, V,
               int(ignore_index), N.stream())
        ctx.save_for_backward(x, lab, lse)
        ctx.ignore_index, ctx.inplace, ctx.shape = ignore_index, inplace_grad, logits.shape
        ctx.mark_non_differentiable(lse)
        return loss.view(label.shape), lse

    @staticmethod
    def backward(ctx, dloss, _dlse):
        x, lab, lse = ctx.saved_tensors
        Nr, V = x.shape
        dx = x if ctx.inplace else torch.empty_like(x)
        dl = _c(dloss.float()).view(-1)
        N.call("pa_softmax_ce_bwd", N.dt(x), N.ptr(x), N.ptr(lab), None, N.ptr(lse), N.ptr(dl), N.ptr(dx),
               Nr, V, int(ctx.ignore_index), 1.0, N.stream())
        return dx.view(ctx.shape), None, None, None


class _SoftmaxCEMeanFn(torch.autograd.Function):
    """CE + mean over the valid labels as ONE node (per-row kernel, then a one-block
    reduce that also counts the valid rows): the scalar loss comes straight out of
    a fused op, so the framework tape can start its reverse pass there."""

    @staticmethod
    def forward(ctx, logits, label, ignore_index, inplace_grad):
        V = logits.shape[-1]
        x = _c(logits).view(-1, V)
        lab = _c(label).view(-1).long()
        Nr = x.shape[0]
        loss = torch.empty(Nr, dtype=torch.float32, device=x.device)
        lse = torch.empty(Nr, dtype=torch.float32, device=x.device)
        N.call("pa_softmax_ce_fwd", N.dt(x), N.ptr(x), N.ptr(lab), None, N.ptr(loss), N.ptr(lse), Nr, V,
               int(ignore_index), N.stream())
        out = torch.empty((), dtype=torch.float32, device=x.device)
        cnt = torch.empty(1, dtype=torch.float32, device=x.device)
        N.call("pa_ce_mean_fwd", N.ptr(loss), N.ptr(lab), Nr, V, int(ignore_index), N.ptr(out), N.ptr(cnt),
               N.stream())
        ctx.save_for_backward(x, lab, lse, cnt)
        ctx.ignore_index, ctx.inplace, ctx.shape = ignore_index, inplace_grad, logits.shape
        return out

    @staticmethod
    def backward(ctx, g):
        x, lab, lse, cnt = ctx.saved_tensors
        Nr, V = x.shape
        dl = torch.empty(Nr, dtype=torch.float32, device=x.device)
        g1 = _c(g.float()).reshape(1)
        N.call("pa_ce_mean_bwd_rows", N.ptr(g1), N.ptr(cnt), N.ptr(dl), Nr, N.stream())
        dx = x if ctx.inplace else torch.empty_like(x)
        N.call("pa_softmax_ce_bwd", N.dt(x), N.ptr(x), N.ptr(lab), None, N.ptr(lse), N.ptr(dl), N.ptr(dx),
               Nr, V, int(ctx.ignore_index), 1.0, N.stream())
        return dx.view(ctx.shape), None, None, None


def softmax_cross_entropy(logits, label, ignore_index=-100, reduction="mean", inplace_grad=False):
    """Fused log-softmax + NLL over the last axis.  loss is fp32."""
    if logits.is_cuda and reduction == "mean":
        return _tape.apply(_SoftmaxCEMeanFn, logits, label, ignore_index, inplace_grad)
    if logits.is_cuda:
        loss, _ = _tape.apply(_SoftmaxCEFn, logits, label, ignore_index, inplace_grad)
    else:
        loss = cross_entropy_tokens(logits, label, ignore_index)
    if reduction == "none":
        return loss
    if reduction == "sum":
        return loss.sum()
    return mean_valid(loss, label, ignore_index)


class _SoftmaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, log):
        V = x.shape[-1]
        x2 = _c(x).view(-1, V)
        y = torch.empty_like(x2)
        N.call("pa_softmax_fwd", N.dt(x2), N.ptr(x2), N.ptr(y), x2.shape[0], V, int(log), N.stream())
        ctx.save_for_backward(y)
        ctx.log = log
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        V = y.shape[-1]
        dy2 = _c(dy).view(-1, V)
        dx = torch.empty_like(y)
        N.call("pa_softmax_bwd", N.dt(y), N.ptr(y), N.ptr(dy2), N.ptr(dx), y.shape[0], V, int(ctx.log), N.stream())
        return dx.view(dy.shape), None


def softmax(x, axis=-1, log=False):
    if x.is_cuda and (axis == -1 or axis == x.dim() - 1) and x.dtype in (torch.float32, torch.bfloat16):
        return _tape.apply(_SoftmaxFn, x, log)
    return torch.log_softmax(x, axis) if log else torch.softmax(x, axis)


# ====================================================================== embedding


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, weight, padding_idx):
        ids_ = _c(ids).view(-1).long()
        H = weight.shape[1]
        out = torch.empty(ids_.numel(), H, dtype=weight.dtype, device=weight.device)
        N.call("pa_embedding_fwd", N.dt(weight), N.ptr(ids_), N.ptr(weight), N.ptr(out), ids_.numel(), H,
               int(padding_idx), N.stream())
        ctx.save_for_backward(ids_)
        ctx.wshape, ctx.wdtype, ctx.pad = weight.shape, weight.dtype, padding_idx
        ctx.weight = weight if getattr(weight, "_pa_main_grad", None) is not None else None
        return out.view(*ids.shape, H)

    @staticmethod
    def backward(ctx, dout):
        (ids_,) = ctx.saved_tensors
        H = ctx.wshape[1]
        d = _c(dout).view(-1, H)
        w = ctx.weight
        mg = getattr(w, "_pa_main_grad", None) if w is not None else None
        if mg is not None and mg.dtype == torch.float32:
            # scatter-add straight into the fp32 main_grad (zeroed first on the first
            # write after zero_grad), like the fused linear's dW epilogue
            if getattr(w, "_pa_grad_fresh", False):
                _oplib_fill(mg, 0.0)
                w._pa_grad_fresh = False
            N.call("pa_embedding_bwd", N.dt(d), N.ptr(ids_), N.ptr(d), N.ptr(mg), ids_.numel(), H, int(ctx.pad),
                   N.stream())
            return None, None, None
        dW = torch.zeros(ctx.wshape, dtype=torch.float32, device=d.device)
        N.call("pa_embedding_bwd", N.dt(d), N.ptr(ids_), N.ptr(d), N.ptr(dW), ids_.numel(), H, int(ctx.pad), N.stream())
        return None, dW.to(ctx.wdtype), None


def embedding(ids, weight, padding_idx=None):
    param_ready(weight)
    pad = -1 if padding_idx is None else int(padding_idx)
    if weight.is_cuda and weight.shape[1] % 8 == 0:
        return _tape.apply(_EmbeddingFn, ids, weight, pad)
    return _tape.apply(_EmbeddingRefFn, ids, weight, pad)


class _EmbeddingRefFn(torch.autograd.Function):
    """Host embedding lookup; dW is a row scatter-add (the padding row gets none)."""

    @staticmethod
    def forward(ctx, ids, w, pad):
        ctx.save_for_backward(ids)
        ctx.meta = (w.shape, w.dtype, pad)
        return w[ids.long()]

    @staticmethod
    def backward(ctx, g):
        (ids,) = ctx.saved_tensors
        shape, dt, pad = ctx.meta
        idx = ids.reshape(-1).long()
        gf = g.reshape(-1, shape[1]).float()
        if pad >= 0:
            gf = gf * (idx != pad).unsqueeze(1)
        dw = torch.zeros(shape, dtype=torch.float32, device=g.device).index_add_(0, idx, gf)
        return None, dw.to(dt), None


# ====================================================================== transpose


def transpose2d(x):
    """out = x.T (contiguous) for a 2-D (or batched 3-D: last two dims) tensor.
    bf16/fp16 on the GPU run the LDS-tiled HIP kernel (csrc/kernels/transpose.hip)."""
    if x.is_cuda and x.dtype in (torch.bfloat16, torch.float16) and x.shape[-1] % 8 == 0 \
            and x.shape[-2] % 8 == 0 and x.stride(-1) == 1 and x.stride(-2) % 8 == 0:
        R, C = x.shape[-2], x.shape[-1]
        if x.dim() == 2:
            out = torch.empty(C, R, device=x.device, dtype=x.dtype)
            N.call("pa_transpose2d", 1, N.ptr(x), N.ptr(out), R, C, x.stride(0), R, 1, 0, 0, N.stream())
            return out
        if x.dim() == 3 and (x.stride(0) % 8 == 0):
            out = torch.empty(x.shape[0], C, R, device=x.device, dtype=x.dtype)
            N.call("pa_transpose2d", 1, N.ptr(x), N.ptr(out), R, C, x.stride(1), R, x.shape[0], x.stride(0),
                   R * C, N.stream())
            return out
    return x.transpose(-1, -2).contiguous()


# dW = X^T dY through the K-inner ("NT") GEMM form on transposed copies; see
# csrc/kernels/transpose.hip for why.  Off on CPU (no effect on numerics).
_DW_VIA_TRANSPOSE = True
_DW_KMAJ = os.environ.get("PADDLE_AMD_DW_KMAJ", "0") == "1"  # MN x MN dW = transposes + K x K (profiles/r3_dw_mn_vs_kmajor_bench_ab.txt); no transposed copies


def _dw_nt_ok(x2, dy2):
    # measured (benchmarks/dw_transpose.py, profiles/r1_dw_transpose.jsonl): the NT form
    # saves more than the two transposes cost unless X is much wider than dY (down_proj)
    return (_DW_VIA_TRANSPOSE and x2.is_cuda and x2.dtype == torch.bfloat16 and dy2.dtype == torch.bfloat16
            and x2.shape[0] % 8 == 0 and x2.shape[1] % 8 == 0 and dy2.shape[1] % 8 == 0
            and x2.shape[0] >= 1024 and x2.shape[1] <= dy2.shape[1])


# Forward y = x W through the NT form as well: a transposed copy W^T of each weight
# is kept next to it and refreshed lazily when the weight changes (optimizer steps
# bump the epoch; plain in-place torch updates bump the tensor version).
_FWD_VIA_WT = True
_WEIGHT_EPOCH = [0]


def bump_weight_epoch():
    """Call after writing parameters through raw pointers (fused optimizers, all-gathers)."""
    _WEIGHT_EPOCH[0] += 1


def _weight_t(w, tokens):
    if not (_FWD_VIA_WT and w.is_cuda and w.dtype == torch.bfloat16 and w.dim() == 2 and tokens >= 1024
            and w.shape[0] % 8 == 0 and w.shape[1] % 8 == 0):
        return None
    key = (_WEIGHT_EPOCH[0], w._version, w.data_ptr())
    wt = getattr(w, "_pa_wt", None)
    if wt is None or getattr(w, "_pa_wt_key", None) != key:
        with torch.no_grad():
            wt = transpose2d(w.detach())
        w._pa_wt, w._pa_wt_key = wt, key
    return wt


# ====================================================================== linear


def _bias_act_bwd(dy2, z2=None):
    """(dZ, db) for Z = XW + b [-> gelu]: ``pa_bias_act_bwd`` computes dZ = dY * gelu'(Z)
    (if ``z2``) and the bias gradient in one pass over dY; returns dZ = dY without z2."""
    Nr, H = dy2.shape
    G = int(N.lib().pa_bias_grad_blocks(Nr, H))
    part = _ws(G * H, dy2.device)
    db = torch.empty(H, dtype=dy2.dtype, device=dy2.device)
    dz = torch.empty_like(dy2) if z2 is not None else dy2
    N.call("pa_bias_act_bwd", N.dt(dy2), int(z2 is not None), N.ptr(dy2), N.ptr(z2),
           N.ptr(dz) if z2 is not None else None, N.ptr(db), N.ptr(part), Nr, H, N.stream())
    return dz, db


def _fast_bias_ok(t):
    return t.is_cuda and t.dtype in (torch.bfloat16, torch.float32) and t.shape[-1] % 8 == 0


def _gelu_tanh(z):
    if _fast_bias_ok(z) and z.is_contiguous():
        g = torch.empty_like(z)
        N.call("pa_gelu_fwd", N.dt(z), N.ptr(z), N.ptr(g), z.numel(), N.stream())
        return g
    return F.gelu(z, approximate="tanh")


def _linear_fwd(x, w, b):
    """x W (+ b).  On the GPU: the hand-written MFMA GEMM (ops/gemm.py) with the
    bias in its epilogue; torch only for shapes that kernel does not cover."""
    K, Nn = w.shape
    x2 = x.reshape(-1, K)
    if _G.supported(x2.shape[0], Nn, K, x2, w):
        # a K-major copy W^T (refreshed once per optimizer step, reused by every
        # micro-batch) lets the forward run the both-K-major form, 6-11 % faster
        # than transposed LDS reads of W (profiles/r2_gemm_v4_sched_ab.jsonl)
        wt = _weight_t(w, x2.shape[0])
        if wt is not None:
            y = _G.gemm(x2, wt, x2.shape[0], Nn, K, a_kmaj=True, b_kmaj=True, bias=b)
        else:
            y = _G.linear_fwd(x2, w, b)
        return y.view(*x.shape[:-1], Nn)
    wt = _weight_t(w, x.numel() // max(x.shape[-1], 1))
    wm = wt.t() if wt is not None else w
    if b is None:
        return torch.matmul(x, wm)
    return torch.addmm(b, x2, wm).view(*x.shape[:-1], wm.shape[-1])


def _acc_mm(acc, a, b):
    """acc += a @ b; ``acc`` may be fp32 while a, b are bf16 (fp32 main_grad):
    one GEMM with an fp32 accumulator, never rounded through bf16."""
    if acc.dtype == a.dtype:
        acc.addmm_(a, b)
    elif acc.is_cuda:
        acc.add_(torch.mm(a, b, out_dtype=acc.dtype))
    else:
        acc.add_(a.to(acc.dtype) @ b.to(acc.dtype))


_DW_SIDE = {}
_DW_PENDING = set()
# Off by default: measured 26.7k -> 13.9k tok/s on LLaMA-7B (gpurun_out/r2_bench_pagemm4):
# two 132-KiB-LDS GEMMs contend for CUs and record_stream() delays frees.
_DW_SIDE_ENABLED = os.environ.get("PADDLE_AMD_DW_STREAM", "0") == "1"


def _dw_side_stream(dev):
    if not (_DW_SIDE_ENABLED and dev.type == "cuda"):
        return None
    s = _DW_SIDE.get(dev)
    if s is None:
        s = _DW_SIDE[dev] = torch.cuda.Stream(device=dev)
    return s


def join_dw_streams(device=None):
    """Make the current stream wait for every dW GEMM issued on the side stream
    (call before reading main_grad: optimizer step, gradient reduce-scatter)."""
    if not _DW_PENDING:
        return
    for dev in list(_DW_PENDING):
        if device is None or dev == device:
            torch.cuda.current_stream(dev).wait_stream(_DW_SIDE[dev])
            _DW_PENDING.discard(dev)


def _linear_bwd(ctx, x, w, dy, need_dx, need_dw):
    K, Nn = w.shape
    dy2 = _c(dy).reshape(-1, Nn)
    x2 = x.reshape(-1, K)
    mg = getattr(w, "_pa_main_grad", None)
    if _G.supported(dy2.shape[0], Nn, K, dy2, w, x2):
        # dX = dY W^T (both K-major), dW = X^T dY (both MN-major) straight from the
        # stored layouts; dW accumulates into the fp32 main_grad in the epilogue
        dx = _G.linear_dx(dy2, w).view(x.shape) if need_dx else None
        dw = None
        if need_dw:
            if mg is not None:
                # the first write after zero_grad() overwrites (no zero fill, no read)
                fresh = getattr(w, "_pa_grad_fresh", False)
                w._pa_grad_fresh = False
                side = _dw_side_stream(w.device)
                if side is None and _DW_KMAJ and x2.shape[0] >= 1024:
                    # dW = X^T dY as a K-major x K-major GEMM over transposed copies:
                    # the kernel's K-major form runs ~1.3x the MN-major (tr_b16) form,
                    # far more than the two transposes cost
                    _G.gemm(transpose2d(_c(x2)), transpose2d(dy2), K, Nn, x2.shape[0], a_kmaj=True, b_kmaj=True,
                            out=mg, accumulate=not fresh)
                elif side is None and x2.shape[0] >= 1024 and Nn >= 2 * K:
                    # dY much wider than X (qkv, gate_up): transpose only X and run the
                    # mixed form -- 3-8 % under the both-MN-major form at these shapes
                    # (profiles/r3_gemm_dw_forms.jsonl), the transpose included
                    _G.gemm(transpose2d(_c(x2)), dy2, K, Nn, x2.shape[0], a_kmaj=True, b_kmaj=False, out=mg,
                            accumulate=not fresh)
                elif side is None:
                    _G.linear_dw(x2, dy2, out=mg, accumulate=not fresh)
                else:
                    # dW is a leaf of the backward graph: run it on a side stream so it
                    # fills the CUs the dX chain leaves idle (partial last rounds of
                    # 688/1376-tile dW grids, launch gaps); readers of main_grad join
                    # the side stream first (join_dw_streams)
                    side.wait_stream(torch.cuda.current_stream(w.device))
                    with torch.cuda.stream(side):
                        _G.linear_dw(x2, dy2, out=mg, accumulate=not fresh)
                    x2.record_stream(side)
                    dy2.record_stream(side)
                    if not _DW_PENDING:
                        # everything after this backward pass sees finished dW
                        torch.autograd.Variable._execution_engine.queue_callback(join_dw_streams)
                    _DW_PENDING.add(w.device)
            else:
                dw = _G.linear_dw(x2, dy2, out=torch.empty(K, Nn, dtype=w.dtype, device=w.device))
        return dx, dw
    dx = torch.matmul(dy, w.t()) if need_dx else None
    dw = None
    if need_dw:
        if _dw_nt_ok(x2, dy2):
            # X^T materialised token-inner, dY as is: the "NN" form, which measured
            # faster than both TN and (X^T, dY^T) NT once the dY transpose is paid
            xa, dyb = transpose2d(_c(x2)), dy2
        else:
            xa, dyb = x2.t(), dy2
        if mg is not None:
            # the engine's post-accumulate hook still fires for w (grad None)
            if getattr(w, "_pa_grad_fresh", False):
                mg.zero_()
                w._pa_grad_fresh = False
            _acc_mm(mg, xa, dyb)
        else:
            dw = torch.matmul(xa, dyb)
    return dx, dw


class _LinearFn(torch.autograd.Function):
    """y = x W (+ b) with W in Paddle's [in, out] layout.

    If the weight carries ``_pa_main_grad`` (a view into a flat gradient buffer
    owned by the sharded DP engine), the weight-gradient GEMM accumulates straight
    into it (the native GEMM's fp32 accumulate epilogue: dW += x^T dy, one
    rounding; the first write after zero_grad overwrites); the engine's
    post-accumulate-grad hook still fires for w, so bucket readiness is unchanged
    -- no temporary dW, no separate accumulate kernel.  The bias is added in the
    GEMM epilogue and its gradient is one HIP column reduction (``pa_bias_act_bwd``).
    """

    @staticmethod
    def forward(ctx, x, w, b):
        y = _linear_fwd(x, w, b)
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx, dw = _linear_bwd(ctx, x, w, dy, ctx.needs_input_grad[0], ctx.needs_input_grad[1])
        db = None
        if ctx.has_b and ctx.needs_input_grad[2]:
            dy2 = dy.reshape(-1, dy.shape[-1])
            if _fast_bias_ok(dy2):
                _, db = _bias_act_bwd(_c(dy2))
            else:
                db = dy2.sum(0).to(dy.dtype)
        return dx, dw, db


class _LinearGeluFn(torch.autograd.Function):
    """g = gelu_tanh(x W + b): bias in the GEMM epilogue, GELU in one HIP pass;
    backward computes dZ = dG * gelu'(Z) and db together (``pa_bias_act_bwd``),
    then the dX / dW GEMMs consume dZ."""

    @staticmethod
    def forward(ctx, x, w, b):
        z = _linear_fwd(x, w, b)
        g = _gelu_tanh(z)
        ctx.save_for_backward(x, w, z)
        return g

    @staticmethod
    def backward(ctx, dg):
        x, w, z = ctx.saved_tensors
        H = z.shape[-1]
        dg2 = _c(dg).reshape(-1, H)
        z2 = z.reshape(-1, H)
        if _fast_bias_ok(dg2) and dg2.dtype == z2.dtype:
            dz2, db = _bias_act_bwd(dg2, _c(z2))
        else:
            # analytic tanh-GELU derivative (no autograd on the host path)
            zf = z2.float()
            c = math.sqrt(2.0 / math.pi)
            t = torch.tanh(c * (zf + 0.044715 * zf.pow(3)))
            dgelu = 0.5 * (1 + t) + 0.5 * zf * (1 - t * t) * c * (1 + 3 * 0.044715 * zf * zf)
            dz2 = (dg2.float() * dgelu).to(dg2.dtype)
            db = dz2.sum(0).to(dg.dtype)
        dz = dz2.view(z.shape)
        dx, dw = _linear_bwd(ctx, x, w, dz, ctx.needs_input_grad[0], ctx.needs_input_grad[1])
        return dx, dw, (db if ctx.needs_input_grad[2] else None)


def linear_gelu(x, weight, bias):
    """gelu(x W + b, approximate='tanh') as one fused autograd node."""
    param_ready(weight)
    param_ready(bias)
    return _tape.apply(_LinearGeluFn, x, weight, bias)


def linear(x, weight, bias=None):
    param_ready(weight)
    if bias is not None:
        param_ready(bias)
    return _tape.apply(_LinearFn, x, weight, bias)


# ====================================================================== tied head
class _LinearTFn(torch.autograd.Function):
    """y = x W^T with W stored [out, in] (a tied embedding table used as the LM head).

    GPU: the hand-written GEMM in all three forms (forward both K-major; dX with W
    MN-major; dW = dY^T X with both operands MN-major, into the fp32 main_grad when
    the table has one).  A vocabulary that is not a multiple of 8 (GPT's 50,257) runs
    the same forms on 8-aligned row buffers (``gemm_padded``): the logits are
    computed into [T, round8(V)] rows and the incoming gradient is laid into
    zero-padded rows, so no product leaves the MFMA kernel."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        V, H = w.shape
        x2 = x.reshape(-1, H)
        if _G.supported(x2.shape[0], 8, H, x2, w) and V >= 8:
            Vp = (V + 7) // 8 * 8
            if Vp == V:
                return _G.gemm(x2, w, x2.shape[0], V, H, a_kmaj=True, b_kmaj=True).view(*x.shape[:-1], V)
            buf = torch.empty(x2.shape[0], Vp, dtype=x.dtype, device=x.device)
            _G.gemm_padded(x2, w, x2.shape[0], V, H, a_kmaj=True, b_kmaj=True, out=buf)
            out = torch.empty(x2.shape[0], V, dtype=x.dtype, device=x.device)
            _copy_native(out, buf[:, :V])
            return out.view(*x.shape[:-1], V)
        return torch.matmul(x, w.t())

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        V, H = w.shape
        x2 = x.reshape(-1, H)
        dy2 = _c(dy).reshape(-1, V)
        need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        mg = getattr(w, "_pa_main_grad", None)
        if V % 8 and V >= 8 and _G.supported(x2.shape[0], H, 8, x2, w):
            # ragged vocabulary: the gradient in zero-padded 8-aligned rows, then the
            # padded GEMM forms (padding enters the K / M extents as zeros)
            T, Vp = x2.shape[0], (V + 7) // 8 * 8
            dyp = torch.empty(T, Vp, dtype=dy2.dtype, device=dy2.device)
            _fill_native(dyp[:, V:], 0.0)
            _copy_native(dyp[:, :V], dy2)
            dx = None
            if need_x:
                dx = torch.empty(T, H, dtype=x.dtype, device=x.device)
                _G.gemm_padded(dyp, w, T, H, V, a_kmaj=True, b_kmaj=False, out=dx)
                dx = dx.view(x.shape)
            dw = None
            if need_w:
                if mg is not None:
                    fresh = getattr(w, "_pa_grad_fresh", False)
                    w._pa_grad_fresh = False
                    _G.gemm_padded(dyp, x2, V, H, T, a_kmaj=False, b_kmaj=False, out=mg, accumulate=not fresh)
                else:
                    g32 = torch.empty(V, H, dtype=torch.float32, device=x.device)
                    _G.gemm_padded(dyp, x2, V, H, T, a_kmaj=False, b_kmaj=False, out=g32)
                    dw = g32.to(w.dtype)
            return dx, dw
        if V % 8 == 0 and _G.supported(x2.shape[0], H, V, x2, w, dy2):
            dx = _G.gemm(dy2, w, x2.shape[0], H, V, a_kmaj=True, b_kmaj=False).view(x.shape) if need_x else None
            dw = None
            if need_w:
                if mg is not None:
                    fresh = getattr(w, "_pa_grad_fresh", False)
                    w._pa_grad_fresh = False
                    _G.gemm(dy2, x2, V, H, x2.shape[0], a_kmaj=False, b_kmaj=False, out=mg, accumulate=not fresh)
                else:
                    dw = _G.gemm(dy2, x2, V, H, x2.shape[0], a_kmaj=False, b_kmaj=False,
                                 out_dtype=torch.float32).to(w.dtype)
            return dx, dw
        dx = torch.matmul(dy2, w).view(x.shape) if need_x else None
        dw = None
        if need_w:
            g = torch.matmul(dy2.t().to(torch.float32) if mg is not None else dy2.t(), x2.to(
                torch.float32) if mg is not None else x2)
            if mg is not None:
                if getattr(w, "_pa_grad_fresh", False):
                    mg.zero_()
                    w._pa_grad_fresh = False
                mg.add_(g)
            else:
                dw = g.to(w.dtype)
        return dx, dw


def linear_t(x, weight):
    """x @ weight^T for a [out, in] weight (tied LM heads), as one fused tape op."""
    param_ready(weight)
    return _tape.apply(_LinearTFn, x, weight)
