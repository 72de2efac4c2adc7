"""Grouped (ragged) SwiGLU expert MLP on the hand-written MFMA GEMM.

All local experts of an MoE layer run as THREE kinds of grouped GEMM launches
instead of one GEMM chain per expert (launch-bound at 64 experts x ~768 rows) or
a padded batched GEMM (wasted rows, a scatter and a gather):

* forward  ``h = x_g @ gate_up[g]``, ``y = swiglu(h)_g @ down[g]`` -- grp_mode 1:
  group g owns rows ``[off[g], off[g+1])`` of the expert-sorted token matrix and of
  the output; each workgroup reads ``off[g]`` / ``off[g+1]`` and masks its tile
  rows, so no padding and no copies.
* backward dX -- the same ragged-row launch with the weights read K-major.
* backward dW -- grp_mode 2: ``dW[g] (+)= x_g^T dY_g``, a per-group reduction over
  the group's rows, accumulated in fp32 straight into the sharded optimizer's
  ``main_grad`` (the same contract as ``ops.linear``).

The reference has no MoE; the per-expert loop it would imply is
``MoELayer`` with a list of experts (distributed/fleet/moe.py).
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _native as N
from . import accum as _accum
from ..autograd import tape as _tape
from . import fp8 as _F8
from . import gemm as _G


def _c(t):
    return t if t.is_contiguous() else t.contiguous()


def supported(x, gate_up, down) -> bool:
    if not (x.is_cuda and _G.enabled() and x.dtype == torch.bfloat16 and x.dim() == 2):
        return False
    if gate_up.dtype != x.dtype or down.dtype != x.dtype or gate_up.dim() != 3 or down.dim() != 3:
        return False
    H, I2 = gate_up.shape[1:]
    return H % 8 == 0 and I2 % 16 == 0 and tuple(down.shape[1:]) == (I2 // 2, H) \
        and gate_up.is_contiguous() and down.is_contiguous()


def _wgrad(w, a, b, offs):
    """Per-expert weight gradient into the main_grad view (or a fresh tensor)."""
    mg = getattr(w, "_pa_main_grad", None)
    if mg is not None:
        # the first write after zero_grad() overwrites (beta = 0): no zero fill
        fresh = getattr(w, "_pa_grad_fresh", False)
        w._pa_grad_fresh = False
        _G.grouped_dw(a, b, offs, out=mg, accumulate=not fresh)
        return None
    return _G.grouped_dw(a, b, offs, out=torch.empty_like(w), accumulate=False)


class _GroupedSwiGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gate_up, down, offs):
        x = _c(x)
        R, H = x.shape
        I2 = gate_up.shape[2]
        I = I2 // 2
        h = torch.empty(R, I2, dtype=x.dtype, device=x.device)
        _G.grouped_rows(x, gate_up, offs, b_kmaj=False, out=h)
        a = torch.empty(R, I, dtype=x.dtype, device=x.device)
        N.call("pa_swiglu_fwd", N.dt(h), N.ptr(h), N.ptr(a), R, I, N.stream())
        y = torch.empty(R, H, dtype=x.dtype, device=x.device)
        _G.grouped_rows(a, down, offs, b_kmaj=False, out=y)
        ctx.save_for_backward(x, gate_up, down, offs, h, a)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, gate_up, down, offs, h, a = ctx.saved_tensors
        dy = _c(dy)
        R, H = x.shape
        I = a.shape[1]
        # da = dy down[g]^T: down[g] is [I, H] = [n][k], read K-major
        da = torch.empty(R, I, dtype=x.dtype, device=x.device)
        _G.grouped_rows(dy, down, offs, b_kmaj=True, out=da)
        dh = torch.empty_like(h)
        N.call("pa_swiglu_bwd", N.dt(h), N.ptr(h), N.ptr(da), N.ptr(dh), R, I, N.stream())
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(R, H, dtype=x.dtype, device=x.device)
            _G.grouped_rows(dh, gate_up, offs, b_kmaj=True, out=dx)
        r = _expert_wgrads(gate_up, down, x, dh, a, dy, offs, False,
                           (ctx.needs_input_grad[1], ctx.needs_input_grad[2]))
        if r is not None:
            return dx, r[0], r[1], None
        d_down = _wgrad(down, a, dy, offs) if ctx.needs_input_grad[2] else None
        d_gu = _wgrad(gate_up, x, dh, offs) if ctx.needs_input_grad[1] else None
        return dx, d_gu, d_down, None


# fp8 expert weight gradients (FLAGS_fp8_wgrad=1; default bf16 x bf16 as the dense
# layers): dW_g = X_g^T dY_g with X and dY quantised per (expert, channel) over the
# expert's tokens and transposed token-contiguous by fp8.hip (pa_f8_group_quant_t),
# then the block-scaled fp8 MFMA in its grouped-K mode (grp_mode 2), fp32 += into
# main_grad.  Measured no faster per micro-batch (profiles/r5_moe_fp8_wgrad_NEGATIVE.md):
# at ~1.5k tokens per expert the tile time is the fp32 main_grad read-modify-write
# of the epilogue, not the MFMA loop.
_F8_WGRAD = os.environ.get("FLAGS_fp8_wgrad", "0") not in ("0", "false", "False")


def _ptrs(ts):
    return (ctypes.c_void_p * len(ts))(*[N.ptr(t) for t in ts])


def _cat_offsets(offs_list, G):
    """Concatenated expert layout of several micro-batches: cum [(n+1) * G] (tokens
    of expert g before micro-batch j) and 64-aligned image columns poffs [G+1]."""
    n = len(offs_list)
    dev = offs_list[0].device
    cum = torch.empty((n + 1) * G, dtype=torch.int32, device=dev)
    poffs = torch.empty(G + 1, dtype=torch.int32, device=dev)
    N.call("pa_group_cat_offsets", n, _ptrs(offs_list), G, N.ptr(cum), N.ptr(poffs), N.stream())
    return cum, poffs


def _image(xs, offs_list, cum, poffs, G, quant):
    """Transposed token-contiguous image [C, ldq] of the experts' rows of every
    micro-batch (e4m3 + per-(expert, channel) scales, or bf16)."""
    xs = [_c(x) for x in xs]
    R, C = sum(x.shape[0] for x in xs), xs[0].shape[1]
    ldq = (R + 64 * G + 63) // 64 * 64
    dev = xs[0].device
    q = torch.empty(C, ldq, dtype=_F8._FP8 if quant else torch.bfloat16, device=dev)
    sc = amax = None
    if quant:
        sc = torch.empty(G, C, dtype=torch.float32, device=dev)
        amax = torch.empty(G, C, dtype=torch.float32, device=dev)
    ld = (ctypes.c_long * len(xs))(*[x.stride(0) for x in xs])
    N.call("pa_group_image", int(quant), len(xs), _ptrs(xs), ld, _ptrs(offs_list), N.ptr(cum), N.ptr(poffs), G, R, C,
           N.ptr(amax), N.ptr(q), ldq, N.ptr(sc), N.stream())
    return q, sc, ldq


def _image_ok(*ts):
    return all(t.shape[1] % 64 == 0 and t.dtype == torch.bfloat16 for t in ts)


def _wgrad_images(w, a_list, b_list, offs_list, G, fp8):
    """dW_g = sum_j a_j[g]^T b_j[g] over the micro-batches j ([G, M, N]) as ONE grouped
    GEMM over the K-major images: into main_grad (overwrite on the step's first
    write, else +=) or a fresh fp32 tensor (returned in w's dtype)."""
    cum, poffs = _cat_offsets(offs_list, G)
    qa, sa, ldq = _image(a_list, offs_list, cum, poffs, G, fp8)
    qb, sb, _ = _image(b_list, offs_list, cum, poffs, G, fp8)
    M, Nn = a_list[0].shape[1], b_list[0].shape[1]
    mg = getattr(w, "_pa_main_grad", None)
    if mg is not None:
        fresh = getattr(w, "_pa_grad_fresh", False)
        w._pa_grad_fresh = False
        out, acc, ret = mg, not fresh, None
    else:
        out, acc = torch.empty(G, M, Nn, dtype=torch.float32, device=qa.device), False
        ret = out
    if fp8:
        rc = N.lib().pa_gemm_f8(1, N.ptr(qa), N.ptr(qb), N.ptr(out), N.ptr(sa), N.ptr(sb), M, Nn, ldq, ldq, ldq, Nn,
                                0, M * Nn, G, 1.0, int(acc), N.ptr(poffs), 2, N.stream())
        if rc != 0:
            raise RuntimeError(f"pa_gemm_f8 (grouped dW) failed rc={rc} G={G} M={M} N={Nn}")
    else:
        _G.gemm(qa, qb, M, Nn, ldq, a_kmaj=True, b_kmaj=True, out=out[0], accumulate=acc, batch=G, sA=0, sB=0,
                sC=out.stride(0), ldc=out.stride(1), grp=poffs, grp_mode=2)
    return None if ret is None else ret.to(w.dtype)


def _wgrad_f8_ok(a, b):
    return _F8_WGRAD and _F8._FP8 is not None and _image_ok(a, b)


def _wgrad_f8(w, a, b, offs, G):
    """Per-expert dW_g = a_g^T b_g ([G, M, N] fp32) on the fp8 grouped-K GEMM."""
    return _wgrad_images(w, [a], [b], [offs], G, True)


# ---- expert dW over all micro-batches of a step (ops/accum.py)
# key: id(gate_up) -> [(gate_up, down, x, dh, a, dy, offs, fp8)] of the deferred
# micro-batches; each entry holds the operands of one micro-batch's two dW GEMMs
_STASH = {}
_MAX_MB = 8  # csrc/kernels/fp8.hip kMaxMb
_DEFER_ON = os.environ.get("FLAGS_defer_expert_wgrad", "1") not in ("0", "false", "False")


def _defer_ok(gate_up, down, x, dh, a, dy):
    return (_DEFER_ON and getattr(gate_up, "_pa_main_grad", None) is not None
            and getattr(down, "_pa_main_grad", None) is not None and _image_ok(x, dh, a, dy))


def _expert_wgrads(gate_up, down, x, dh, a, dy, offs, fp8, needs):
    """The two expert dW of one micro-batch: deferred while accum.deferring(), else
    computed over every deferred micro-batch plus this one in one GEMM each.
    Returns (d_gate_up, d_down), or None when the regular per-micro-batch path
    applies (nothing deferred, or no main_grad to accumulate into)."""
    if not _defer_ok(gate_up, down, x, dh, a, dy):
        return None
    key = id(gate_up)
    lst = _STASH.get(key, [])
    if lst and lst[0][0] is not gate_up:  # a stale entry of a freed layer that reused the id
        _STASH.pop(key, None)
        lst = []
    if _accum.deferring() and len(lst) < _MAX_MB - 1:
        _STASH.setdefault(key, []).append((gate_up, down, x, dh, a, dy, offs, fp8))
        return None, None
    if not lst:
        return None
    _STASH.pop(key, None)
    return _flush_entries(lst + [(gate_up, down, x, dh, a, dy, offs, fp8)], needs)


def _flush_entries(ents, needs=(True, True)):
    gate_up, down = ents[0][0], ents[0][1]
    G = gate_up.shape[0]
    fp8 = _F8_WGRAD and ents[0][7] and _F8._FP8 is not None
    offs = [e[6] for e in ents]
    d_down = _wgrad_images(down, [e[4] for e in ents], [e[5] for e in ents], offs, G, fp8) if needs[1] else None
    d_gu = _wgrad_images(gate_up, [e[2] for e in ents], [e[3] for e in ents], offs, G, fp8) if needs[0] else None
    return d_gu, d_down


def _flush_all():
    """Deferred experts whose last micro-batch never came (accum.flush)."""
    while _STASH:
        _, ents = _STASH.popitem()
        _flush_entries(ents)


_accum.register_flush(_flush_all)
_accum.register_discard(_STASH.clear)


class _F8Weights:
    """fp8 copies of one expert weight stack [G, K, N]: K-major per-output-channel
    for the forward (B = W^T) and row-quantised as stored for the dX GEMM."""

    def __init__(self):
        self.fwd = _F8.VersionedCache(_F8.quant_cols_t)
        self.bwd = _F8.VersionedCache(lambda w: _F8.quant_rows(w.reshape(-1, w.shape[-1])))


def _f8_cache(w):
    c = getattr(w, "_pa_f8_grouped", None)
    if c is None:
        c = w._pa_f8_grouped = _F8Weights()
    return c


def _rows_f8(a, bq, sb, offs, N_, out):
    """out[rows_g] = a[rows_g] @ B_g^T with B_g = bq[g] ([N_, K] e4m3, scales sb[g])."""
    aq, sa = _F8.quant_rows(a)
    G = sb.numel() // N_
    if G and a.shape[0] > 0:
        _F8.gemm_f8(aq, sa, bq, sb, a.shape[0], N_, a.shape[1], out=out, batch=G, sB=N_ * a.shape[1], grp=offs,
                    grp_mode=1)
    return out


class _GroupedSwiGLUF8Fn(torch.autograd.Function):
    """fp8 e4m3 forward and dX GEMMs (block-scaled MFMA, per-token and per-channel
    scales); the weight gradients stay bf16 x bf16 -> fp32 main_grad."""

    @staticmethod
    def forward(ctx, x, gate_up, down, offs):
        x = _c(x)
        R, H = x.shape
        G, _, I2 = gate_up.shape
        I = I2 // 2
        gq, gs = _f8_cache(gate_up).fwd.get(gate_up)  # [G, 2I, H]
        dq, ds = _f8_cache(down).fwd.get(down)        # [G, H, I]
        h = _rows_f8(x, gq, gs, offs, I2, torch.empty(R, I2, dtype=x.dtype, device=x.device))
        a = torch.empty(R, I, dtype=x.dtype, device=x.device)
        N.call("pa_swiglu_fwd", N.dt(h), N.ptr(h), N.ptr(a), R, I, N.stream())
        y = _rows_f8(a, dq, ds, offs, H, torch.empty(R, H, dtype=x.dtype, device=x.device))
        ctx.save_for_backward(x, gate_up, down, offs, h, a)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, gate_up, down, offs, h, a = ctx.saved_tensors
        dy = _c(dy)
        R, H = x.shape
        I = a.shape[1]
        dbq, dbs = _f8_cache(down).bwd.get(down)      # [G*I, H]: B = down[g] as [I][H]
        da = _rows_f8(dy, dbq, dbs, offs, I, torch.empty(R, I, dtype=x.dtype, device=x.device))
        dh = torch.empty_like(h)
        N.call("pa_swiglu_bwd", N.dt(h), N.ptr(h), N.ptr(da), N.ptr(dh), R, I, N.stream())
        dx = None
        if ctx.needs_input_grad[0]:
            gbq, gbs = _f8_cache(gate_up).bwd.get(gate_up)  # [G*H, 2I]: B = gate_up[g] as [H][2I]
            dx = _rows_f8(dh, gbq, gbs, offs, H, torch.empty(R, H, dtype=x.dtype, device=x.device))
        G = gate_up.shape[0]
        r = _expert_wgrads(gate_up, down, x, dh, a, dy, offs, True,
                           (ctx.needs_input_grad[1], ctx.needs_input_grad[2]))
        if r is not None:
            return dx, r[0], r[1], None
        if _wgrad_f8_ok(x, dh) and _wgrad_f8_ok(a, dy):
            d_down = _wgrad_f8(down, a, dy, offs, G) if ctx.needs_input_grad[2] else None
            d_gu = _wgrad_f8(gate_up, x, dh, offs, G) if ctx.needs_input_grad[1] else None
            return dx, d_gu, d_down, None
        d_down = _wgrad(down, a, dy, offs) if ctx.needs_input_grad[2] else None
        d_gu = _wgrad(gate_up, x, dh, offs) if ctx.needs_input_grad[1] else None
        return dx, d_gu, d_down, None


def supported_f8(x, gate_up, down) -> bool:
    H, I2 = gate_up.shape[1:]
    return supported(x, gate_up, down) and H % 16 == 0 and I2 % 32 == 0 and _F8._FP8 is not None


def expert_offsets(counts, device, total_rows):
    """Row offsets + tile table (``gemm.group_table``) from per-expert row counts (a
    device tensor -- no host sync -- or host ints)."""
    if torch.is_tensor(counts):
        offs = torch.zeros(counts.numel() + 1, dtype=torch.int32, device=device)
        offs[1:] = torch.cumsum(counts, 0)
    else:
        import itertools

        offs = torch.tensor([0, *itertools.accumulate(counts)], dtype=torch.int32).to(device, non_blocking=True)
    return _G.group_table(offs, total_rows)


def grouped_swiglu_mlp(x, gate_up, down, counts, fp8=False):
    """``x``: [R, H] tokens sorted by expert, ``counts``: rows per expert (device
    tensor or host ints, sum R); ``gate_up`` [G, H, 2I], ``down`` [G, I, H].  Returns
    [R, H].  ``fp8``: forward and dX GEMMs in e4m3 (weights quantised once per
    optimizer step)."""
    offs = expert_offsets(counts, x.device, x.shape[0])
    fn = _GroupedSwiGLUF8Fn if fp8 else _GroupedSwiGLUFn
    return _tape.apply(fn, x, gate_up, down, offs)
