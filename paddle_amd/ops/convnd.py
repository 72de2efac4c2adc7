"""Channel-first (NCHW / NCDHW) conv, transposed conv, pooling, unpool and maxout
on the gfx950 kernels of ``csrc/kernels/convnd.hip`` -- the GPU kernels behind the
Fluid ``conv2d`` / ``conv3d`` / ``conv2d_transpose`` / ``conv3d_transpose`` /
``pool2d`` / ``pool3d`` / ``max_pool{2,3}d_with_index`` / ``unpool`` / ``maxout``
operators (the reference runs these on cuDNN or math/{im2col,vol2col,pooling}.cu).

Convolution is vol2col + an exact-fp32 MFMA GEMM (``pa_sgemm``) per chunk of
images (chunks bound the column buffer), groups on the GEMM's second batch
dimension; dgrad is W^T dY + col2vol (gather, no atomics); wgrad sums
dY col^T over the images of a chunk with float-atomic accumulation into fp32.
Transposed convolution reuses the same three pieces with the roles swapped.
bf16 / fp16 inputs are computed in fp32 and cast back (the NHWC bf16 model path
lives in :mod:`paddle_amd.ops.conv`).

Reference: operators/conv_cudnn_op.cu.cc:43-171, conv_transpose_cudnn_op.cu.cc,
math/vol2col.cu, math/im2col.cu, math/pooling.cu:25-1037, math/maxouting.cu,
math/unpooling.cu, pool_op.cc (output sizes), unpool_op.cc.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _native as N
from ..autograd import tape as _tape  # noqa: E402

_ENABLED = os.environ.get("PADDLE_AMD_CONVND", "1") != "0"
_COL_BUDGET = 1 << 28  # floats per column chunk (1 GiB)
# 2-D implicit GEMM (B gathered in the tile loader, no column buffer): correct but
# measured slower than vol2col + the vectorised GEMM on Fluid ResNet-50 (58.8 vs
# 45.1 ms of kernel time per step, profiles/r2_fluid_resnet50_fp32_ab.jsonl) -- the
# per-element index decomposition costs more than the column round trip; kept as the
# zero-extra-memory option.
_IMPLICIT = os.environ.get("PADDLE_AMD_CONV_IMPLICIT", "0") == "1"
_DT = {torch.float32: 0, torch.bfloat16: 1}


def enabled():
    return _ENABLED


def set_enabled(flag: bool):
    global _ENABLED
    _ENABLED = bool(flag)


def _ok(x):
    return _ENABLED and x.is_cuda and x.dtype in (torch.float32, torch.bfloat16, torch.float16)


def _tup(v, nd):
    if isinstance(v, (list, tuple)):
        v = [int(t) for t in v]
        return tuple(v if len(v) == nd else v * nd if len(v) == 1 else v[:nd])
    return (int(v),) * nd


def _arr(vals):
    a = (ctypes.c_int * len(vals))(*[int(v) for v in vals])
    return a


class deterministic:
    """Within the block every exact-fp32 GEMM (``pa_sgemm``) reduces split-K slices
    through per-slice slabs summed in a fixed order instead of float atomics, so its
    result does not depend on workgroup completion order.  Process-wide default:
    ``FLAGS_cudnn_deterministic=1`` (the reference's determinism flag)."""

    def __init__(self, on=True):
        self.on, self.prev = int(bool(on)), None

    def __enter__(self):
        L = N.lib()
        self.prev = int(L.pa_sgemm_get_deterministic())
        if self.prev != self.on:
            L.pa_sgemm_set_deterministic(self.on)
        return self

    def __exit__(self, *exc):
        if self.prev != self.on:
            N.lib().pa_sgemm_set_deterministic(self.prev)


def sgemm(A, sam, sak, B, sbk, sbn, C, ldc, M, Nn, K, Z1=1, Z2=1, bs1=(0, 0, 0), bs2=(0, 0, 0), kb=1,
          kbA=0, kbB=0, bias=None, bs_bias2=0, alpha=1.0, beta=0.0, atomic=False, conv=None):
    """Strided batched fp32 GEMM: C[z](m, n) = alpha * sum_b A[z, b](m, :) B[z, b](:, n) (+ bias[m] | + beta C)."""
    if Z1 * Z2 > 65535:
        raise ValueError("sgemm: batch too large")
    N.call("pa_sgemm", N.ptr(A), sam, sak, N.ptr(B), sbk, sbn, N.ptr(C), ldc, M, Nn, K, int(Z1), int(Z2),
           bs1[0], bs1[1], bs1[2], bs2[0], bs2[1], bs2[2], int(kb), kbA, kbB, N.ptr(bias), bs_bias2, float(alpha),
           float(beta), int(bool(atomic)), _arr(conv) if conv is not None else None, N.stream())


def _geo(C, sp, osp, k, s, p, d):
    return _arr([C, *sp, *osp, *k, *s, *p, *d])


def _vol2col(x, nb, geo, rows, S):
    col = torch.empty(nb, rows, S, dtype=x.dtype, device=x.device)
    N.call("pa_vol2col", _DT[x.dtype], N.ptr(x), N.ptr(col), geo, int(nb), N.stream())
    return col


def _col2vol(col, x, nb, geo, accumulate=False):
    N.call("pa_col2vol", N.ptr(col), N.ptr(x), geo, int(nb), int(accumulate), N.stream())


def _chunk(n, per_img, groups):
    nb = max(1, min(n, _COL_BUDGET // max(per_img, 1)))
    return max(1, min(nb, 65535 // max(groups, 1)))


def _pad3(t):
    return (1,) * (3 - len(t)) + tuple(t)


def _pad3z(t):
    return (0,) * (3 - len(t)) + tuple(t)


def out_size(i, k, s, p, d):
    return (i + 2 * p - d * (k - 1) - 1) // s + 1


# ------------------------------------------------------------------ convolution


def _pointwise(k, s, p):
    """1x1(x1) kernel, stride 1, no padding: the column matrix of an image IS the
    image ([C][S]), so vol2col / col2vol are skipped (most ResNet bottleneck convs)."""
    return all(v == 1 for v in k) and all(v == 1 for v in s) and all(v == 0 for v in p)


def _conv_geo(sp, osp, k, s, p, d):
    """implicit-GEMM geometry for pa_sgemm: H, W, OW, kh, kw, sh, sw, ph, pw, dh, dw."""
    return [sp[0], sp[1], osp[1], k[0], k[1], s[0], s[1], p[0], p[1], d[0], d[1]]


def _geo2(geo):
    """(H, W, OW, kh, kw, sh, sw, ph, pw, dh, dw) of a 2-D geo array, or None for 3-D."""
    v = list(geo)
    if v[1] != 1 or v[4] != 1 or v[7] != 1:
        return None
    return [v[2], v[3], v[6], v[8], v[9], v[11], v[12], v[14], v[15], v[17], v[18]]


def _pw_geo(geo):
    """geo = (C, D, H, W, OD, OH, OW, kd, kh, kw, sd, sh, sw, pd, ph, pw, dd, dh, dw)."""
    v = list(geo)
    return v[7:10] == [1, 1, 1] and v[10:13] == [1, 1, 1] and v[13:16] == [0, 0, 0]


_COL_KEEP = int(os.environ.get("PADDLE_AMD_CONV_COL_CACHE_MB", "4096")) << 20  # bytes per conv


def _conv_fwd(x, w, b, s, p, d, G, keep=None):
    Nn, C = x.shape[0], x.shape[1]
    sp = tuple(x.shape[2:])
    nd = len(sp)
    Cout = w.shape[0]
    k = tuple(w.shape[2:])
    osp = tuple(out_size(sp[i], k[i], s[i], p[i], d[i]) for i in range(nd))
    KT = 1
    for v in k:
        KT *= v
    S = 1
    for v in osp:
        S *= v
    Cg, Coutg = C // G, Cout // G
    CgK = Cg * KT
    geo = _geo(C, _pad3(sp), _pad3(osp), _pad3(k), _pad3(s), _pad3z(p), _pad3(d))
    y = torch.empty((Nn, Cout) + osp, dtype=torch.float32, device=x.device)
    wc = w.contiguous()
    if _IMPLICIT and len(sp) == 2 and not _pointwise(k, s, p) and Nn * G <= 65535:
        # 2-D: implicit GEMM, B gathered from the image in the tile loader (no column buffer)
        H, W = sp
        sgemm(wc, CgK, 1, x, 0, 1, y, S, Coutg, S, CgK, Z1=Nn, Z2=G,
              bs1=(0, C * H * W, Cout * S), bs2=(Coutg * CgK, Cg * H * W, Coutg * S), bias=b, bs_bias2=Coutg,
              conv=_conv_geo(sp, osp, k, s, p, d))
        return y, geo, osp
    if _pointwise(k, s, p):
        if Nn * G > 65535:
            raise ValueError("conv: batch x groups too large")
        sgemm(wc, CgK, 1, x, S, 1, y, S, Coutg, S, CgK, Z1=Nn, Z2=G,
              bs1=(0, C * S, Cout * S), bs2=(Coutg * CgK, CgK * S, Coutg * S), bias=b, bs_bias2=Coutg)
        return y, geo, osp
    nb = _chunk(Nn, C * KT * S, G)
    for n0 in range(0, Nn, nb):
        m = min(nb, Nn - n0)
        col = _vol2col(x[n0:n0 + m], m, geo, C * KT, S)
        sgemm(wc, CgK, 1, col, S, 1, y[n0:n0 + m], S, Coutg, S, CgK, Z1=m, Z2=G,
              bs1=(0, C * KT * S, Cout * S), bs2=(Coutg * CgK, CgK * S, Coutg * S), bias=b, bs_bias2=Coutg)
        if keep is not None:
            keep.append(col)
    if keep is not None and sum(c.numel() * 4 for c in keep) > _COL_KEEP:
        keep.clear()
    return y, geo, osp


def _conv_dgrad(dy, w, x_shape, geo, G):
    Nn, C = x_shape[0], x_shape[1]
    Cout = w.shape[0]
    KT = w[0, 0].numel()
    S = dy[0, 0].numel()
    Cg, Coutg = C // G, Cout // G
    CgK = Cg * KT
    dx = torch.empty(x_shape, dtype=torch.float32, device=dy.device)
    if KT == 1 and _pw_geo(geo):  # pointwise: W^T dY lands in dx directly
        sgemm(w, 1, CgK, dy, S, 1, dx, S, CgK, S, Coutg, Z1=Nn, Z2=G,
              bs1=(0, Cout * S, C * S), bs2=(Coutg * CgK, Coutg * S, CgK * S))
        return dx
    nb = _chunk(Nn, C * KT * S, G)
    for n0 in range(0, Nn, nb):
        m = min(nb, Nn - n0)
        col = torch.empty(m, C * KT, S, dtype=torch.float32, device=dy.device)
        sgemm(w, 1, CgK, dy[n0:n0 + m], S, 1, col, S, CgK, S, Coutg, Z1=m, Z2=G,
              bs1=(0, Cout * S, C * KT * S), bs2=(Coutg * CgK, Coutg * S, CgK * S))
        _col2vol(col, dx[n0:n0 + m], m, geo)
    return dx


def _conv_wgrad(dy, x, w_shape, geo, G, cols=None):
    Nn, C = x.shape[0], x.shape[1]
    Cout = w_shape[0]
    KT = 1
    for v in w_shape[2:]:
        KT *= v
    S = dy[0, 0].numel()
    Cg, Coutg = C // G, Cout // G
    CgK = Cg * KT
    dw = torch.zeros(w_shape, dtype=torch.float32, device=dy.device)
    g2 = _geo2(geo)
    if _IMPLICIT and g2 is not None and not (KT == 1 and _pw_geo(geo)):
        # 2-D: dW[g] = sum_img dY[img][g] col(x[img])[g]^T with col gathered in the
        # loader; images on the k-batch, split over workgroups by the launcher
        H, W = g2[0], g2[1]
        sgemm(dy, S, 1, x, 1, 0, dw, CgK, Coutg, CgK, S, Z1=1, Z2=G,
              bs2=(Coutg * S, Cg * H * W, Coutg * CgK), kb=Nn, kbA=Cout * S, kbB=C * H * W, atomic=True, conv=g2)
        return dw
    nb = _chunk(Nn, C * KT * S, G)
    pw = KT == 1 and _pw_geo(geo)
    for ci, n0 in enumerate(range(0, Nn, nb)):
        m = min(nb, Nn - n0)
        if pw:
            col = x[n0:n0 + m]
        elif cols:  # the forward's column chunks (same chunking)
            col = cols[ci]
        else:
            col = _vol2col(x[n0:n0 + m], m, geo, C * KT, S)
        # dW[g] += sum_img dY[img][g] col[img][g]^T  (float atomics across chunks / splits)
        # (images on the kernel's k-batch; the launcher splits k-batch / K over
        # workgroups when the dW grid is small)
        sgemm(dy[n0:n0 + m], S, 1, col, 1, S, dw, CgK, Coutg, CgK, S, Z1=1, Z2=G,
              bs2=(Coutg * S, CgK * S, Coutg * CgK), kb=m, kbA=Cout * S, kbB=C * KT * S, atomic=True)
    return dw


def _bias_grad(dy):
    Nn, C = dy.shape[0], dy.shape[1]
    S = dy[0, 0].numel()
    db = torch.empty(C, dtype=torch.float32, device=dy.device)
    N.call("pa_chan_sum", N.ptr(dy), N.ptr(db), Nn, C, S, 0, N.stream())
    return db


class _ConvNdFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, s, p, d, G):
        dt = x.dtype
        xf, wf = x.float().contiguous(), w.float().contiguous()
        bf = b.float().contiguous() if b is not None else None
        keep = [] if ctx.needs_input_grad[1] else None  # column chunks reused by the wgrad
        y, geo, _ = _conv_fwd(xf, wf, bf, s, p, d, G, keep)
        ctx.save_for_backward(xf, wf)
        ctx.cols = keep
        ctx.conf = (geo, G, dt, w.dtype, b is not None)
        return y.to(dt)

    @staticmethod
    def backward(ctx, dy):
        xf, wf = ctx.saved_tensors
        geo, G, dt, wdt, has_b = ctx.conf
        dyf = dy.float().contiguous()
        dx = _conv_dgrad(dyf, wf, tuple(xf.shape), geo, G).to(dt) if ctx.needs_input_grad[0] else None
        dw = _conv_wgrad(dyf, xf, tuple(wf.shape), geo, G, ctx.cols).to(wdt) if ctx.needs_input_grad[1] else None
        ctx.cols = None
        db = _bias_grad(dyf).to(wdt) if has_b and ctx.needs_input_grad[2] else None
        return dx, dw, db, None, None, None, None


def conv_grads(x, w, dy, stride, padding, dilation, groups, need_x=True, need_w=True):
    """Explicit conv data / filter gradients from (x, w, dY) -- the Fluid
    ``conv2d_grad`` op's kernels, with no forward recompute (the column matrix of
    the wgrad is rebuilt by vol2col).  Returns (dx | None, dw | None) in x / w dtypes."""
    nd = x.dim() - 2
    s, p, d = _tup(stride, nd), _tup(padding, nd), _tup(dilation, nd)
    xf, wf = x.float().contiguous(), w.float().contiguous()
    dyf = dy.float().contiguous()
    sp, k = tuple(xf.shape[2:]), tuple(wf.shape[2:])
    osp = tuple(dyf.shape[2:])
    geo = _geo(xf.shape[1], _pad3(sp), _pad3(osp), _pad3(k), _pad3(s), _pad3z(p), _pad3(d))
    G = int(groups)
    dx = _conv_dgrad(dyf, wf, tuple(xf.shape), geo, G).to(x.dtype) if need_x else None
    dw = _conv_wgrad(dyf, xf, tuple(wf.shape), geo, G).to(w.dtype) if need_w else None
    return dx, dw


def supported_conv(x, w, groups=1):
    return (_ok(x) and x.dim() in (4, 5) and w.dim() == x.dim() and groups >= 1 and x.shape[1] % groups == 0
            and w.shape[0] % groups == 0 and w.shape[1] * groups == x.shape[1] and x.numel() > 0)


def conv_nd(x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
    """x [N, C, (D,) H, W], w [Cout, C / groups, (kd,) kh, kw]."""
    nd = x.dim() - 2
    return _tape.apply(_ConvNdFn, x, w, b, _tup(stride, nd), _tup(padding, nd), _tup(dilation, nd), int(groups))


# ------------------------------------------------------------------ transposed convolution


def _convT_fwd(x, w, s, p, d, G, osp):
    Nn, Cin = x.shape[0], x.shape[1]
    sp = tuple(x.shape[2:])
    k = tuple(w.shape[2:])
    Coutg = w.shape[1]
    Cout = Coutg * G
    Cing = Cin // G
    KT = w[0, 0].numel()
    S = x[0, 0].numel()
    CoKT = Coutg * KT
    geo = _geo(Cout, _pad3(osp), _pad3(sp), _pad3(k), _pad3(s), _pad3z(p), _pad3(d))
    y = torch.empty((Nn, Cout) + tuple(osp), dtype=torch.float32, device=x.device)
    nb = _chunk(Nn, Cout * KT * S, G)
    for n0 in range(0, Nn, nb):
        m = min(nb, Nn - n0)
        col = torch.empty(m, Cout * KT, S, dtype=torch.float32, device=x.device)
        sgemm(w, 1, CoKT, x[n0:n0 + m], S, 1, col, S, CoKT, S, Cing, Z1=m, Z2=G,
              bs1=(0, Cin * S, Cout * KT * S), bs2=(Cing * CoKT, Cing * S, CoKT * S))
        _col2vol(col, y[n0:n0 + m], m, geo)
    return y, geo


class _ConvTNdFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, s, p, d, G, osp):
        dt = x.dtype
        xf, wf = x.float().contiguous(), w.float().contiguous()
        y, geo = _convT_fwd(xf, wf, s, p, d, G, osp)
        ctx.save_for_backward(xf, wf)
        ctx.conf = (geo, G, dt, w.dtype)
        return y.to(dt)

    @staticmethod
    def backward(ctx, dy):
        xf, wf = ctx.saved_tensors
        geo, G, dt, wdt = ctx.conf
        dyf = dy.float().contiguous()
        Nn, Cin = xf.shape[0], xf.shape[1]
        Coutg = wf.shape[1]
        Cout, Cing = Coutg * G, Cin // G
        KT = wf[0, 0].numel()
        S = xf[0, 0].numel()
        CoKT = Coutg * KT
        dx = torch.empty(xf.shape, dtype=torch.float32, device=dy.device) if ctx.needs_input_grad[0] else None
        dw = torch.zeros(wf.shape, dtype=torch.float32, device=dy.device) if ctx.needs_input_grad[1] else None
        nb = _chunk(Nn, Cout * KT * S, G)
        for n0 in range(0, Nn, nb):
            m = min(nb, Nn - n0)
            col = _vol2col(dyf[n0:n0 + m], m, geo, Cout * KT, S)
            if dx is not None:  # dx[img][g] = W[g] col(dY)[img][g]
                sgemm(wf, CoKT, 1, col, S, 1, dx[n0:n0 + m], S, Cing, S, CoKT, Z1=m, Z2=G,
                      bs1=(0, Cout * KT * S, Cin * S), bs2=(Cing * CoKT, CoKT * S, Cing * S))
            if dw is not None:  # dW[g] += x[img][g] col(dY)[img][g]^T
                sgemm(xf[n0:n0 + m], S, 1, col, 1, S, dw, CoKT, Cing, CoKT, S, Z1=1, Z2=G,
                      bs2=(Cing * S, CoKT * S, Cing * CoKT), kb=m, kbA=Cin * S, kbB=Cout * KT * S, atomic=True)
        return (dx.to(dt) if dx is not None else None, dw.to(wdt) if dw is not None else None,
                None, None, None, None, None)


def conv_transpose_nd(x, w, stride=1, padding=0, dilation=1, groups=1, output_padding=0):
    """x [N, Cin, (D,) H, W], w [Cin, Cout / groups, (kd,) kh, kw] (Paddle / torch layout)."""
    nd = x.dim() - 2
    s, p, d, op = _tup(stride, nd), _tup(padding, nd), _tup(dilation, nd), _tup(output_padding, nd)
    k = tuple(w.shape[2:])
    osp = tuple((x.shape[2 + i] - 1) * s[i] - 2 * p[i] + d[i] * (k[i] - 1) + 1 + op[i] for i in range(nd))
    return _tape.apply(_ConvTNdFn, x, w, s, p, d, int(groups), osp)


def supported_conv_transpose(x, w, groups=1):
    return (_ok(x) and x.dim() in (4, 5) and w.dim() == x.dim() and x.shape[1] == w.shape[0]
            and x.shape[1] % groups == 0 and x.numel() > 0)


# ------------------------------------------------------------------ pooling


def pool_out(i, k, s, p, ceil):
    return (i - k + 2 * p + s - 1) // s + 1 if ceil else (i - k + 2 * p) // s + 1


class _PoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, typ, k, s, p, exclusive, ceil, need_mask):
        x = x.contiguous()
        dt = x.dtype
        xc = x if dt in _DT else x.float()
        nd = x.dim() - 2
        sp = tuple(x.shape[2:])
        osp = tuple(pool_out(sp[i], k[i], s[i], p[i], ceil) for i in range(nd))
        NC = x.shape[0] * x.shape[1]
        geo = _arr([*_pad3(sp), *_pad3(osp), *_pad3(k), *_pad3(s), *_pad3z(p)])
        y = torch.empty(tuple(x.shape[:2]) + osp, dtype=xc.dtype, device=x.device)
        mask = torch.empty(y.shape, dtype=torch.int32, device=x.device) if typ == 0 else None
        N.call("pa_pool_fwd", _DT[xc.dtype], N.ptr(xc), N.ptr(y), N.ptr(mask), NC, geo, typ, int(exclusive),
               N.stream())
        ctx.save_for_backward(mask)
        ctx.conf = (typ, exclusive, NC, tuple(x.shape), xc.dtype, dt, [*_pad3(sp), *_pad3(osp), *_pad3(k),
                                                                       *_pad3(s), *_pad3z(p)])
        if mask is not None:
            ctx.mark_non_differentiable(mask)
        return y.to(dt), mask

    @staticmethod
    def backward(ctx, dy, _dm):
        (mask,) = ctx.saved_tensors
        typ, exclusive, NC, xshape, cdt, dt, geo = ctx.conf
        dyc = dy.contiguous().to(cdt)
        dx = torch.empty(xshape, dtype=cdt, device=dy.device)
        N.call("pa_pool_bwd", _DT[cdt], N.ptr(dyc), N.ptr(mask), N.ptr(dx), NC, _arr(geo), typ, int(exclusive),
               N.stream())
        return dx.to(dt), None, None, None, None, None, None, None


def supported_pool(x):
    return _ok(x) and x.dim() in (4, 5) and x.numel() > 0


def pool_nd(x, pooling_type="max", ksize=2, stride=None, padding=0, exclusive=True, ceil_mode=False,
            global_pooling=False, return_mask=False):
    """Max / avg pooling over the trailing 2 or 3 dims of an NC[D]HW tensor.
    Returns ``out`` (and the int32 in-plane argmax for max pooling if ``return_mask``)."""
    nd = x.dim() - 2
    k = _tup(ksize, nd)
    s = _tup(stride if stride is not None else ksize, nd)
    p = _tup(padding, nd)
    if global_pooling:
        k, p = tuple(x.shape[2:]), (0,) * nd
    typ = 0 if pooling_type == "max" else 1
    y, mask = _tape.apply(_PoolFn, x, typ, k, s, p, bool(exclusive), bool(ceil_mode), bool(return_mask))
    return (y, mask) if return_mask else y


# ------------------------------------------------------------------ unpool / maxout


class _UnpoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mask, osp):
        x = x.contiguous()
        dt = x.dtype
        xc = x if dt in _DT else x.float()
        m = mask.to(torch.int32).contiguous()
        NC = x.shape[0] * x.shape[1]
        IS, OS = x[0, 0].numel(), 1
        for v in osp:
            OS *= v
        out = torch.zeros(tuple(x.shape[:2]) + tuple(osp), dtype=xc.dtype, device=x.device)
        bad = torch.zeros(1, dtype=torch.int32, device=x.device)
        N.call("pa_unpool", _DT[xc.dtype], 0, N.ptr(xc), N.ptr(m), N.ptr(out), NC, IS, OS, N.ptr(bad), N.stream())
        if int(bad.item()):
            raise ValueError("unpool: an index is outside the output plane")
        ctx.save_for_backward(m)
        ctx.conf = (tuple(x.shape), NC, IS, OS, xc.dtype, dt)
        return out.to(dt)

    @staticmethod
    def backward(ctx, dout):
        (m,) = ctx.saved_tensors
        xshape, NC, IS, OS, cdt, dt = ctx.conf
        d = dout.contiguous().to(cdt)
        dx = torch.empty(xshape, dtype=cdt, device=dout.device)
        N.call("pa_unpool", _DT[cdt], 1, N.ptr(d), N.ptr(m), N.ptr(dx), NC, IS, OS, None, N.stream())
        return dx.to(dt), None, None


def unpool2d(x, indices, ksize, strides, paddings):
    """Max unpool (unpool_op.cc: out = (in - 1) * stride - 2 * pad + ksize)."""
    k, s, p = _tup(ksize, 2), _tup(strides, 2), _tup(paddings, 2)
    osp = tuple((x.shape[2 + i] - 1) * s[i] - 2 * p[i] + k[i] for i in range(2))
    return _tape.apply(_UnpoolFn, x, indices, osp)


class _MaxoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, groups):
        x = x.contiguous()
        dt = x.dtype
        xc = x if dt in _DT else x.float()
        Nn, C = x.shape[0], x.shape[1]
        Co = C // groups
        S = x[0, 0].numel()
        y = torch.empty((Nn, Co) + tuple(x.shape[2:]), dtype=xc.dtype, device=x.device)
        N.call("pa_maxout", _DT[xc.dtype], N.ptr(xc), None, None, N.ptr(y), Nn, Co, groups, S, N.stream())
        ctx.save_for_backward(xc, y)
        ctx.conf = (groups, dt)
        return y.to(dt)

    @staticmethod
    def backward(ctx, dy):
        xc, y = ctx.saved_tensors
        groups, dt = ctx.conf
        d = dy.contiguous().to(xc.dtype)
        dx = torch.empty_like(xc)
        Nn, Co = y.shape[0], y.shape[1]
        N.call("pa_maxout", _DT[xc.dtype], N.ptr(xc), N.ptr(y), N.ptr(d), N.ptr(dx), Nn, Co, groups,
               y[0, 0].numel(), N.stream())
        return dx.to(dt), None


def maxout(x, groups):
    if x.shape[1] % groups:
        raise ValueError("maxout: channels must be divisible by groups")
    return _tape.apply(_MaxoutFn, x, int(groups))


# ------------------------------------------------------------------ batch norm (channel-first)


def _bn_part(x, C):
    M = x.numel() // C
    G = int(N.lib().pa_bn_nchw_groups(C, M))
    return torch.empty(C * G * 2, dtype=torch.float32, device=x.device)


class _BatchNormNCHW(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, scale, bias, run_mean, run_var, momentum, eps, training, relu, unbiased):
        x = x.contiguous()
        dt = x.dtype
        xc = x if dt in _DT else x.float()
        Nn, C = x.shape[0], x.shape[1]
        S = x[0, 0].numel() if x.dim() > 2 else 1
        f = lambda t: t.float().contiguous() if t is not None else None  # noqa: E731
        sc, bi, rm, rv = f(scale), f(bias), f(run_mean), f(run_var)
        y = torch.empty_like(xc)
        mean = torch.empty(C, dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        mean_out = torch.empty_like(mean) if training else rm.clone()
        var_out = torch.empty_like(mean) if training else rv.clone()
        part = _bn_part(xc, C)
        N.call("pa_bn_nchw_fwd", _DT[xc.dtype], N.ptr(xc), N.ptr(y), N.ptr(sc), N.ptr(bi), N.ptr(rm), N.ptr(rv),
               N.ptr(mean_out), N.ptr(var_out), N.ptr(mean), N.ptr(rstd), N.ptr(part), Nn, C, S, float(eps),
               float(momentum), int(training), int(relu), int(unbiased), N.stream())
        ctx.save_for_backward(xc, y, mean, rstd, sc)
        ctx.conf = (relu, dt, scale.dtype if scale is not None else None, bias.dtype if bias is not None else None,
                    Nn, C, S)
        ctx.mark_non_differentiable(mean_out, var_out, mean, rstd)
        return y.to(dt), mean_out, var_out, mean, rstd

    @staticmethod
    def backward(ctx, dy, *_):
        xc, y, mean, rstd, sc = ctx.saved_tensors
        relu, dt, sdt, bdt, Nn, C, S = ctx.conf
        d = dy.contiguous().to(xc.dtype)
        dscale = torch.empty(C, dtype=torch.float32, device=dy.device)
        dbias = torch.empty_like(dscale)
        dx = torch.empty_like(xc) if ctx.needs_input_grad[0] else None
        N.call("pa_bn_nchw_bwd", _DT[xc.dtype], N.ptr(xc), N.ptr(d), N.ptr(y), N.ptr(mean), N.ptr(rstd), N.ptr(sc),
               N.ptr(dscale), N.ptr(dbias), N.ptr(dx), N.ptr(_bn_part(xc, C)), Nn, C, S, int(relu), N.stream())
        return (dx.to(dt) if dx is not None else None, dscale.to(sdt) if sdt is not None else None,
                dbias.to(bdt) if bdt is not None else None, None, None, None, None, None, None, None)


def supported_bn(x):
    return _ok(x) and x.dim() >= 2 and x.numel() > 0 and x.is_contiguous()


def batch_norm_nchw(x, scale, bias, run_mean, run_var, momentum=0.9, eps=1e-5, training=True, relu=False,
                    unbiased_running_var=False):
    """Channel-first BatchNorm (Fluid batch_norm, NCHW / NC / NCDHW).
    Returns (y, mean_out, var_out, saved_mean, saved_inv_std); running averages use
    the biased batch variance (Fluid batch_norm_op.cc; ``unbiased_running_var`` for the
    2.x layer convention) and Paddle's momentum (running = m * running + (1 - m) * batch)."""
    return _tape.apply(_BatchNormNCHW, x, scale, bias, run_mean, run_var, float(momentum), float(eps), bool(training),
                                bool(relu), bool(unbiased_running_var))
