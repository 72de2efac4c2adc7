"""NHWC bf16 convolution, batch norm and pooling on the hand-written gfx950 kernels.

* conv2d forward: implicit GEMM (csrc/kernels/gemm.hip ``pa_conv_gemm``: the MFMA
  GEMM with an NHWC gather of the A operand; padding/edges are zero-filled by the
  buffer range check).  Input channels not a multiple of 64 (the 3-channel stem)
  take an explicit im2col (``pa_im2col_nhwc``) + the plain GEMM.
* conv2d dgrad: the same implicit GEMM over dY with the flipped, transposed kernel
  and a zero-insertion factor = stride (power of two), i.e. no col2im scatter.
* conv2d wgrad: dW = dY^T im2col(X) with both operands MN-major (1x1 / stride-1
  convs read X directly); fp32 output.
* batch norm: shifted fp32 sums per block + fp64 finalize; optional fused ReLU
  (the backward masks dY with the saved output).
* max pool: argmax byte per element, gather backward; global average pool.

Reference behaviour: paddle/fluid/operators/conv_cudnn_op.cu.cc:43-171,
batch_norm_op.cu.cc:170, math/pooling.cu:25-189, math/im2col.cu.
``supported_*`` decide eligibility; callers use the torch path only for shapes or
dtypes these kernels do not cover.
"""
from __future__ import annotations

import math
import os

import torch

from . import _native as _nat
from . import gemm as _G
from ..autograd import tape as _tape  # noqa: E402


_ENABLED = [True]


def set_enabled(flag: bool):
    """Route NHWC conv / BN / pool to the native kernels (True) or to ATen (False)."""
    _ENABLED[0] = bool(flag)


def _i(v):
    return int(v)


def _pair(v):
    return tuple(v) if isinstance(v, (list, tuple)) else (v, v)


def _pow2(v):
    return v > 0 and (v & (v - 1)) == 0


def supported_conv(x, w, stride, padding, dilation, groups):
    if not (_ENABLED[0] and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and groups == 1 and _G.enabled()):
        return False
    if not x.is_contiguous():
        return False
    N, H, W, C = x.shape
    Cout = w.shape[0]
    sy, sx = _pair(stride)
    if Cout % 8 or not (_pow2(sy) and _pow2(sx)):
        return False
    if isinstance(padding, str):
        return False
    return True


def _out_hw(H, W, KH, KW, s, p, d):
    return (H + 2 * p[0] - d[0] * (KH - 1) - 1) // s[0] + 1, (W + 2 * p[1] - d[1] * (KW - 1) - 1) // s[1] + 1


def _im2col(x, KH, KW, s, p, d, OH, OW, Kp):
    N, H, W, C = x.shape
    col = torch.empty(N * OH * OW, Kp, dtype=x.dtype, device=x.device)
    _nat.call("pa_im2col_nhwc", _nat.ptr(x), _nat.ptr(col), N, H, W, C, OH, OW, KH, KW, s[0], s[1], p[0], p[1],
              d[0], d[1], Kp, _nat.stream())
    return col


# output-channel counts up to this take the 64-wide tile kernel (csrc/kernels/convsn.hip)
_SN_MAX = [int(os.environ.get("FLAGS_conv_sn_max_cout", "128"))]


def _sn(x, wk, y, bias, geo, stats=None, acc=False):
    """pa_conv_sn (64-channel tiles; optional BN statistics of y into ``stats``;
    ``acc``: y += conv)."""
    N, OH, OW, Cout = y.shape
    part = shift = None
    G = 0
    if stats is not None:
        G = int(_nat.lib().pa_conv_sn_tiles(N * OH * OW))
        part = torch.empty(G * 2 * Cout, dtype=torch.float32, device=y.device)
        shift = stats.get("shift")
    rc = _nat.lib().pa_conv_sn_acc(_nat.ptr(x), _nat.ptr(wk), _nat.ptr(y), _nat.ptr(bias), *geo, _nat.ptr(part),
                                   _nat.ptr(shift), int(acc), _nat.stream())
    if rc == 0 and stats is not None:
        stats["part"], stats["G"] = part, G
    return rc == 0


def _conv_fwd(x, w, b, s, p, d, stats=None):
    N, H, W, C = x.shape
    Cout, _, KH, KW = w.shape
    OH, OW = _out_hw(H, W, KH, KW, s, p, d)
    K = KH * KW * C
    wk = w.to(x.dtype).permute(0, 2, 3, 1).reshape(Cout, K)  # [Cout][(kh, kw, c)]
    bias = b.to(x.dtype) if b is not None else None
    if C % 64 == 0:
        wk = wk.contiguous()
        y = torch.empty(N, OH, OW, Cout, dtype=x.dtype, device=x.device)
        geo = (N, H, W, C, OH, OW, Cout, KH, KW, s[0], s[1], p[0], p[1], d[0], d[1], 0, 0)
        if Cout <= _SN_MAX[0] and _sn(x, wk, y, bias, geo, stats):
            return y
        if stats is not None:
            # 256-wide tiles: the same per-tile statistics from the staged epilogue
            G = int(_nat.lib().pa_conv_sn_tiles(N * OH * OW))
            part = torch.empty(G * 2 * Cout, dtype=torch.float32, device=x.device)
            rc = _nat.lib().pa_conv_gemm_stats(_nat.ptr(x), _nat.ptr(wk), _nat.ptr(y), _nat.ptr(bias), *geo, 0,
                                               _nat.ptr(part), _nat.ptr(stats.get("shift")), _nat.stream())
            if rc == 0:
                stats["part"], stats["G"] = part, G
                return y
        rc = _nat.lib().pa_conv_gemm(_nat.ptr(x), _nat.ptr(wk), _nat.ptr(y), _nat.ptr(bias), N, H, W, C, OH, OW,
                                     Cout, KH, KW, s[0], s[1], p[0], p[1], d[0], d[1], 0, 0, _nat.stream())
        _nat.check(rc, "pa_conv_gemm")
        return y
    Kp = (K + 7) // 8 * 8
    col = _im2col(x, KH, KW, s, p, d, OH, OW, Kp)
    wp = torch.zeros(Cout, Kp, dtype=x.dtype, device=x.device)
    wp[:, :K] = wk
    y = _G.gemm(col, wp, N * OH * OW, Cout, Kp, a_kmaj=True, b_kmaj=True, bias=bias)
    return y.view(N, OH, OW, Cout)


def _dgrad_weight(w, dt):
    """wd[c][(kh, kw, co)] = w[co][c][KH-1-kh][KW-1-kw] in ONE strided copy (transpose
    and tap flip as negative strides of the source), cast to ``dt``."""
    Cout, C, KH, KW = w.shape
    if w.dtype not in (torch.float32, torch.bfloat16) or dt not in (torch.float32, torch.bfloat16):
        return w.to(dt).flip(2, 3).permute(1, 2, 3, 0).reshape(C, KH * KW * Cout).contiguous()
    from . import aten_native as _an

    s0, s1, s2, s3 = w.stride()
    out = torch.empty(C, KH, KW, Cout, dtype=dt, device=w.device)
    base = w.data_ptr() + ((KH - 1) * s2 + (KW - 1) * s3) * w.element_size()
    _an.strided_copy(out, base, w.dtype, [s1, -s2, -s3, s0])
    return out.view(C, KH * KW * Cout)


def _bnb_ok(bnb, shape, dt):
    bx = bnb.get("x") if bnb else None
    by = bnb.get("y") if bnb else None
    return (bx is not None and tuple(bx.shape) == tuple(shape) and bx.dtype == dt and bx.is_contiguous()
            and (by is None or (tuple(by.shape) == tuple(shape) and by.dtype == dt and by.is_contiguous())))


def _conv_dgrad(dy, w, x_shape, s, p, d, into=None, bnb=None):
    """dX of the convolution.  ``into``: an exclusively owned gradient of x already
    summed by the engine (e.g. the residual branch's): dX is accumulated into it in
    the GEMM epilogue and ``into`` is returned (no separate add pass).
    ``bnb`` (x is the output of a training BatchNorm, see ``batch_norm_nhwc_train``):
    the epilogue also emits that BN's backward statistics of the final dX; the
    partials are attached as ``dx._pa_bnpart`` (any other in-place write clears it)."""
    N, H, W, C = x_shape
    Cout, _, KH, KW = w.shape
    OH, OW = dy.shape[1], dy.shape[2]
    if Cout % 64 == 0 and C % 8 == 0:
        # dX = conv(zero-inserted dY, flipped W^T): wd[c][kh][kw][co] = w[co][c][KH-1-kh][KW-1-kw]
        wd = _dgrad_weight(w, dy.dtype)
        acc = (into is not None and into.shape == (N, H, W, C) and into.dtype == dy.dtype and into.is_contiguous())
        dx = into if acc else torch.empty(N, H, W, C, dtype=dy.dtype, device=dy.device)
        pyy, pxx = d[0] * (KH - 1) - p[0], d[1] * (KW - 1) - p[1]
        geo = (N, OH, OW, Cout, H, W, C, KH, KW, 1, 1, pyy, pxx, d[0], d[1], int(math.log2(s[0])),
               int(math.log2(s[1])))
        L = _nat.lib()
        if C % 64 == 0 and _bnb_ok(bnb, (N, H, W, C), dy.dtype):
            G = int(L.pa_conv_sn_tiles(N * H * W))
            part = torch.empty(G * 2 * C, dtype=torch.float32, device=dy.device)
            src = (_nat.ptr(part), _nat.ptr(bnb["x"]), _nat.ptr(bnb.get("y")), _nat.ptr(bnb["mean"]),
                   _nat.ptr(bnb["rstd"]), _nat.ptr(bnb.get("w")), _nat.ptr(bnb.get("b")), int(bnb["wdt"]),
                   int(bnb["relu"]))
            if C <= _SN_MAX[0]:
                rc = L.pa_conv_sn_bnbwd(_nat.ptr(dy), _nat.ptr(wd), _nat.ptr(dx), *geo, int(acc), *src,
                                        _nat.stream())
            else:
                rc = L.pa_conv_gemm_bnbwd(_nat.ptr(dy), _nat.ptr(wd), _nat.ptr(dx), None, *geo, int(acc),
                                          src[0], None, *src[1:], _nat.stream())
            if rc == 0:
                dx._pa_bnpart = (part, G, bnb["mean"])
                return dx
        if acc and getattr(into, "_pa_bnpart", None) is not None:
            into._pa_bnpart = None  # its statistics no longer describe the sum
        if C <= _SN_MAX[0] and _sn(dy, wd, dx, None, geo, acc=acc):
            return dx
        rc = L.pa_conv_gemm_acc(_nat.ptr(dy), _nat.ptr(wd), _nat.ptr(dx), None, *geo, int(acc), _nat.stream())
        if rc == 0:
            return dx
    # rare shapes: autograd of the torch convolution
    xs = torch.zeros(N, C, H, W, dtype=dy.dtype, device=dy.device)
    return torch.nn.grad.conv2d_input(xs.shape, w.to(dy.dtype), dy.permute(0, 3, 1, 2), s, p, d).permute(
        0, 2, 3, 1).contiguous()


# weight gradient on the gathered 64x256-tile kernel (convsn.hip): "auto" = when the
# wide path would need an im2col buffer (k > 1 or strided); measured per ResNet-50
# shape in profiles/r4_conv_sn_probe.jsonl (1x1 stride-1 stays on the split-K GEMM)
_WGRAD_SN = [os.environ.get("FLAGS_conv_wgrad_sn", "auto")]


def _wgrad_sn_wanted(C, Cout, KH, KW, s):
    m = _WGRAD_SN[0]
    if m == "0" or C % 64 or Cout % 8:
        return False
    return m == "1" or KH * KW > 1 or s != (1, 1)


def _conv_wgrad(dy, x, w_shape, s, p, d, wdtype=torch.float32):
    """dW in the parameter's layout [Cout, C, KH, KW] (contiguous) and dtype."""
    N, H, W, C = x.shape
    Cout, _, KH, KW = w_shape
    OH, OW = dy.shape[1], dy.shape[2]
    M = N * OH * OW
    K = KH * KW * C
    if _wgrad_sn_wanted(C, Cout, KH, KW, s) and wdtype in (torch.float32, torch.bfloat16):
        L = _nat.lib()
        nws = int(L.pa_conv_wgrad_sn_ws2(N, H, W, C, OH, OW, Cout, KH, KW))
        if nws > 0:
            ws = torch.empty(nws, dtype=torch.float32, device=x.device)
            dw = torch.empty(Cout, C, KH, KW, dtype=wdtype, device=x.device)
            rc = L.pa_conv_wgrad_sn_w(_nat.ptr(dy), _nat.ptr(x), _nat.ptr(dw), int(wdtype == torch.bfloat16),
                                      _nat.ptr(ws), N, H, W, C, OH, OW, Cout, KH, KW, s[0], s[1], p[0], p[1], d[0],
                                      d[1], 0, _nat.stream())
            if rc == 0:
                return dw
    if KH == 1 and KW == 1 and s == (1, 1) and p == (0, 0) and C % 8 == 0:
        col, Kp = x.reshape(M, C), C
    else:
        Kp = (K + 7) // 8 * 8
        col = _im2col(x, KH, KW, s, p, d, OH, OW, Kp)
    dwk = torch.empty(Cout, Kp, dtype=torch.float32, device=x.device)
    # dW[co][k] = sum_m dY[m][co] col[m][k]: both operands stored [m][..] (MN-major);
    # few output tiles, very deep reduction -> split-K across the chip
    _G.gemm_splitk(dy.reshape(M, Cout), col, Cout, Kp, M, a_kmaj=False, b_kmaj=False, out=dwk)
    src = dwk[:, :K].reshape(Cout, KH, KW, C).permute(0, 3, 1, 2)
    if KH == 1 and KW == 1 and wdtype == torch.float32:
        return src.reshape(Cout, C, 1, 1)  # already the parameter layout
    out = torch.empty(Cout, C, KH, KW, dtype=wdtype, device=x.device)
    out.copy_(src)  # one pass: layout + cast
    return out


class _Conv2dNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, s, p, d, stats=None, bnsrc=None):
        y = _conv_fwd(x, w, b, s, p, d, stats)
        ctx.save_for_backward(x, w)
        ctx.conf = (s, p, d, b is not None)
        if bnsrc is not None:
            bnsrc = dict(bnsrc, y=x if bnsrc.get("y_mask") else None)
        ctx.bnsrc = bnsrc if _bnb_ok(bnsrc, x.shape, x.dtype) else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        s, p, d, has_b = ctx.conf
        dy = dy.contiguous()
        into = getattr(ctx, "grad_prev", None)
        into = into[0] if into else None
        dx = (_conv_dgrad(dy, w, tuple(x.shape), s, p, d, into, getattr(ctx, "bnsrc", None))
              if ctx.needs_input_grad[0] else None)
        if dx is not None:
            dx._pa_acc_ok = True  # exclusively owned: later producers may accumulate into it
        dw = _conv_wgrad(dy, x, tuple(w.shape), s, p, d, w.dtype) if ctx.needs_input_grad[1] else None
        db = dy.reshape(-1, dy.shape[-1]).float().sum(0).to(w.dtype) if has_b and ctx.needs_input_grad[2] else None
        return dx, dw, db, None, None, None, None, None


def conv2d_nhwc(x, weight, bias=None, stride=1, padding=0, dilation=1, stats=None):
    """x [N, H, W, C] bf16 contiguous, weight [Cout, Cin, KH, KW] (Paddle layout).
    ``stats`` (a dict, optional): request the BatchNorm batch statistics of the output
    from the conv epilogue (``stats["shift"]``: fp32 [Cout] shift, e.g. the running
    mean, or absent); on return it holds ``part`` / ``G`` when the kernel emitted them
    (64-channel-tile path), for :func:`batch_norm_nhwc_train`'s ``stats``."""
    s, p, d = _pair(stride), _pair(padding), _pair(dilation)
    # x produced by a training BatchNorm (batch_norm_nhwc_train marks its output): the
    # data gradient's epilogue computes that BN's backward statistics
    bnsrc = getattr(x, "_pa_bnsrc", None) if _BNB[0] else None
    return _tape.apply(_Conv2dNHWC, x, weight, bias, tuple(map(_i, s)), tuple(map(_i, p)), tuple(map(_i, d)), stats,
                       bnsrc)


# BatchNorm backward statistics from the consuming conv's data-gradient epilogue.
# Off by default: measured slower end to end (ResNet-50 bs 256: 7,386 vs 7,803
# img/s, profiles/r4_resnet50_prof_bnbwd_NEGATIVE.md) -- the separate bn_reduce pass
# runs at full HBM bandwidth, while the x / y reads added to the dgrad epilogues
# (short-K 1x1 convs: the epilogue is most of the kernel) are not overlapped with
# MFMA work: +4.4 ms/step of epilogue for -2.3 ms/step of bn_reduce.
_BNB = [os.environ.get("FLAGS_conv_bn_bwd_stats", "0") == "1"]


# ------------------------------------------------------------------ depthwise conv (dwconv.hip)


def supported_dwconv(x, w, groups):
    """Depthwise NHWC bf16: groups == C, weight [C * mult, 1, KH, KW], C % 8 == 0."""
    return (_ENABLED[0] and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.is_contiguous()
            and w.dim() == 4 and w.shape[1] == 1 and groups == x.shape[3] and x.shape[3] % 8 == 0
            and w.shape[0] % x.shape[3] == 0)


class _DwConvNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, s, p, d):
        Nn, H, W, C = x.shape
        Cout, _, KH, KW = w.shape
        OH, OW = (H + 2 * p[0] - d[0] * (KH - 1) - 1) // s[0] + 1, (W + 2 * p[1] - d[1] * (KW - 1) - 1) // s[1] + 1
        wb = w.to(torch.bfloat16).reshape(Cout, KH * KW).t().contiguous()  # [taps, Cout] for 16-B loads
        bb = b.to(torch.bfloat16).contiguous() if b is not None else None
        y = torch.empty(Nn, OH, OW, Cout, dtype=torch.bfloat16, device=x.device)
        _nat.call("pa_dwconv_fwd", _nat.ptr(x), _nat.ptr(wb), _nat.ptr(bb), _nat.ptr(y), Nn, H, W, C, Cout, KH, KW, s[0], s[1],
               p[0], p[1], d[0], d[1], _nat.stream())
        ctx.save_for_backward(x, wb)
        ctx.conf = (s, p, d, b is not None, w.dtype, tuple(w.shape))
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wb = ctx.saved_tensors
        s, p, d, has_b, wdt, (Cout, _, KH, KW) = ctx.conf
        dy = dy.contiguous().to(torch.bfloat16)
        Nn, H, W, C = x.shape
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            _nat.call("pa_dwconv_dgrad", _nat.ptr(dy), _nat.ptr(wb), _nat.ptr(dx), Nn, H, W, C, Cout, KH, KW, s[0], s[1], p[0],
                   p[1], d[0], d[1], _nat.stream())
        if ctx.needs_input_grad[1]:
            dw32 = torch.zeros(wb.shape, dtype=torch.float32, device=x.device)  # [taps, Cout]
            _nat.call("pa_dwconv_wgrad", _nat.ptr(dy), _nat.ptr(x), _nat.ptr(dw32), Nn, H, W, C, Cout, KH, KW, s[0], s[1], p[0],
                   p[1], d[0], d[1], _nat.stream())
            dw = dw32.t().reshape(Cout, 1, KH, KW).to(wdt)
        if has_b and ctx.needs_input_grad[2]:
            db = dy.reshape(-1, Cout).float().sum(0).to(wdt)
        return dx, dw, db, None, None, None


def dwconv2d_nhwc(x, weight, bias=None, stride=1, padding=0, dilation=1):
    """Depthwise conv: x [N, H, W, C] bf16, weight [C * mult, 1, KH, KW]."""
    s, p, d = _pair(stride), _pair(padding), _pair(dilation)
    return _tape.apply(_DwConvNHWC, x, weight, bias, tuple(map(_i, s)), tuple(map(_i, p)), tuple(map(_i, d)))


# ------------------------------------------------------------------ batch norm


def supported_bn(x):
    return _ENABLED[0] and x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and x.shape[-1] % 8 == 0 and x.dim() >= 2


def _wdt(w):
    if w is None:
        return 0, None
    if w.dtype == torch.float32:
        return 0, w.contiguous()
    return 1, w.to(torch.bfloat16).contiguous()


class _BatchNormNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, run_mean, run_var, momentum, eps, relu, res, stats=None, link=None):
        C = x.shape[-1]
        rows = x.numel() // C
        wdt, wc = _wdt(w)
        _, bc = _wdt(b) if b is not None else (0, None)
        if b is not None and w is not None and bc.dtype != wc.dtype:
            bc = bc.to(wc.dtype)
        pre = stats is not None and stats.get("part") is not None
        G = 0 if pre else int(_nat.lib().pa_bn_blocks(rows, C))
        part = None if pre else torch.empty(G * 2 * C, dtype=torch.float32, device=x.device)
        mean = torch.empty(C, dtype=torch.float32, device=x.device)
        rstd = torch.empty(C, dtype=torch.float32, device=x.device)
        y = torch.empty_like(x)
        rm = run_mean if (run_mean is not None and run_mean.dtype == torch.float32) else None
        rv = run_var if rm is not None else None
        if pre:
            # statistics already emitted by the producing conv's epilogue
            _nat.call("pa_bn_fwd_stats", _nat.ptr(stats["part"]), int(stats["G"]), _nat.ptr(stats.get("shift")),
                      _nat.ptr(x), _nat.ptr(y), _nat.ptr(wc), _nat.ptr(bc), wdt, _nat.ptr(rm), _nat.ptr(rv),
                      _nat.ptr(mean), _nat.ptr(rstd), rows, C, float(eps), float(momentum), int(relu),
                      _nat.ptr(res), _nat.stream())
        else:
            _nat.call("pa_bn_fwd_train", _nat.ptr(x), _nat.ptr(y), _nat.ptr(wc), _nat.ptr(bc), wdt, _nat.ptr(rm),
                      _nat.ptr(rv), _nat.ptr(mean), _nat.ptr(rstd), _nat.ptr(part), rows, C, float(eps),
                      float(momentum), int(relu), _nat.ptr(res), _nat.stream())
        if (run_mean is not None and rm is None and run_mean.dtype == torch.bfloat16 and run_var is not None
                and run_var.dtype == torch.bfloat16 and run_mean.is_contiguous() and run_var.is_contiguous()):
            # bf16 running stats (a bf16-cast model): one native update launch
            _nat.call("pa_bn_running_update", 1, _nat.ptr(run_mean), _nat.ptr(run_var), _nat.ptr(mean),
                      _nat.ptr(rstd), C, rows, float(eps), float(momentum), _nat.stream())
        elif run_mean is not None and rm is None:  # running stats kept in another dtype: update on the side
            with torch.no_grad():
                var = 1.0 / (rstd.double() ** 2) - eps
                unb = var * rows / max(rows - 1, 1)
                run_mean.mul_(momentum).add_((1 - momentum) * mean.to(run_mean.dtype))
                run_var.mul_(momentum).add_((1 - momentum) * unb.to(run_var.dtype))
        # relu without a residual: backward recomputes the mask from x (y not kept)
        ctx.save_for_backward(x, y if (relu and res is not None) else None, mean, rstd, wc,
                              bc if (relu and res is None) else None)
        ctx.conf = (relu, wdt, w is not None, b is not None, res is not None)
        if link is not None and relu:
            # what a consuming conv's dgrad epilogue needs for this BN's backward sums
            # (no reference to y itself: y carries the link; a residual layer's mask
            # source y is the consuming conv's own input)
            link.update(x=x, y_mask=res is not None, mean=mean, rstd=rstd, w=wc, b=bc, wdt=wdt, relu=1)
        ctx.wdtype = w.dtype if w is not None else None
        ctx.bdtype = b.dtype if b is not None else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, mean, rstd, wc, bc = ctx.saved_tensors
        relu, wdt, has_w, has_b, has_res = ctx.conf
        C = x.shape[-1]
        rows = x.numel() // C
        bp = getattr(dy, "_pa_bnpart", None)
        dy = dy.contiguous()
        coef = torch.empty(3 * C, dtype=torch.float32, device=x.device)
        dw = torch.empty(C, dtype=torch.float32, device=x.device)
        db = torch.empty(C, dtype=torch.float32, device=x.device)
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if has_res else None
        if bp is not None and relu and bp[2].data_ptr() == mean.data_ptr():
            # the reduction came from the epilogue of the conv that produced dy
            _nat.call("pa_bn_bwd_part", _nat.ptr(bp[0]), int(bp[1]), _nat.ptr(x), _nat.ptr(dy), _nat.ptr(y),
                      _nat.ptr(mean), _nat.ptr(rstd), _nat.ptr(wc), _nat.ptr(bc), wdt, _nat.ptr(dx), _nat.ptr(dw),
                      _nat.ptr(db), _nat.ptr(coef), rows, C, int(relu), _nat.ptr(dres), _nat.stream())
        else:
            G = int(_nat.lib().pa_bn_blocks(rows, C))
            part = torch.empty(G * 2 * C, dtype=torch.float32, device=x.device)
            _nat.call("pa_bn_bwd2", _nat.ptr(x), _nat.ptr(dy), _nat.ptr(y), _nat.ptr(mean), _nat.ptr(rstd),
                      _nat.ptr(wc), _nat.ptr(bc), wdt, _nat.ptr(dx), _nat.ptr(dw), _nat.ptr(db), _nat.ptr(coef),
                      _nat.ptr(part), rows, C, int(relu), _nat.ptr(dres), _nat.stream())
        dx._pa_acc_ok = True  # fresh, exclusively owned gradients (see ops.conv._conv_dgrad's into)
        if dres is not None:
            dres._pa_acc_ok = True
        return (dx, dw.to(ctx.wdtype) if has_w else None, db.to(ctx.bdtype) if has_b else None,
                None, None, None, None, None, dres, None, None)


def batch_norm_nhwc_train(x, weight, bias, running_mean, running_var, momentum=0.9, eps=1e-5, relu=False,
                          residual=None, stats=None):
    """Training-mode BatchNorm over all axes but the last (channels), optionally
    fused with a residual add and a ReLU: relu(BN(x) + residual).
    ``momentum``: Paddle convention, running = momentum * running + (1 - momentum) * batch."""
    if residual is not None:
        if not relu:
            raise ValueError("the fused residual form is relu(bn(x) + residual)")
        residual = residual.contiguous()
    link = {} if (relu and _BNB[0]) else None
    y = _tape.apply(_BatchNormNHWC, x, weight, bias, running_mean, running_var, float(momentum), float(eps),
                    bool(relu), residual, stats, link)
    if link:
        y._pa_bnsrc = link  # read by conv2d_nhwc when y feeds a convolution
    return y


def batch_norm_nhwc_eval(x, weight, bias, running_mean, running_var, eps=1e-5, relu=False):
    C = x.shape[-1]
    mean = running_mean.float().contiguous()
    rstd = torch.rsqrt(running_var.float() + eps).contiguous()
    wdt, wc = _wdt(weight)
    _, bc = _wdt(bias) if bias is not None else (0, None)
    if bc is not None and wc is not None and bc.dtype != wc.dtype:
        bc = bc.to(wc.dtype)
    if torch.is_grad_enabled() and (x.requires_grad or (weight is not None and weight.requires_grad)):
        # differentiable eval-mode BN (rare): plain torch expression
        sh = mean.to(x.dtype), rstd.to(x.dtype)
        y = (x - sh[0]) * sh[1]
        if weight is not None:
            y = y * weight.to(x.dtype)
        if bias is not None:
            y = y + bias.to(x.dtype)
        return torch.relu(y) if relu else y
    y = torch.empty_like(x)
    _nat.call("pa_bn_apply", _nat.ptr(x), _nat.ptr(y), _nat.ptr(mean), _nat.ptr(rstd), _nat.ptr(wc), _nat.ptr(bc),
              wdt, x.numel() // C, C, int(relu), _nat.stream())
    return y


# --------------------------------------------------------------------- pooling


class _MaxPoolNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        N, H, W, C = x.shape
        OH = (H + 2 * p[0] - k[0]) // s[0] + 1
        OW = (W + 2 * p[1] - k[1]) // s[1] + 1
        y = torch.empty(N, OH, OW, C, dtype=x.dtype, device=x.device)
        idx = torch.empty(N, OH, OW, C, dtype=torch.uint8, device=x.device)
        _nat.call("pa_maxpool_nhwc_fwd", _nat.ptr(x), _nat.ptr(y), _nat.ptr(idx), N, H, W, C, OH, OW, k[0], k[1],
                  s[0], s[1], p[0], p[1], _nat.stream())
        ctx.save_for_backward(idx)
        ctx.conf = (x.shape, k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        (N, H, W, C), k, s, p = ctx.conf
        dy = dy.contiguous()
        dx = torch.empty(N, H, W, C, dtype=dy.dtype, device=dy.device)
        _nat.call("pa_maxpool_nhwc_bwd", _nat.ptr(dy), _nat.ptr(idx), _nat.ptr(dx), N, H, W, C, dy.shape[1],
                  dy.shape[2], k[0], k[1], s[0], s[1], p[0], p[1], _nat.stream())
        return dx, None, None, None


def supported_pool(x, ceil_mode=False):
    return (_ENABLED[0] and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.is_contiguous() and x.shape[-1] % 8 == 0
            and not ceil_mode)


def max_pool2d_nhwc(x, kernel_size, stride=None, padding=0):
    k = tuple(map(_i, _pair(kernel_size)))
    s = tuple(map(_i, _pair(stride if stride is not None else kernel_size)))
    p = tuple(map(_i, _pair(padding)))
    return _tape.apply(_MaxPoolNHWC, x, k, s, p)


class _GapNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        N, H, W, C = x.shape
        y = torch.empty(N, 1, 1, C, dtype=x.dtype, device=x.device)
        _nat.call("pa_gap_nhwc_fwd", _nat.ptr(x), _nat.ptr(y), N, H * W, C, _nat.stream())
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        N, H, W, C = ctx.shape
        dy = dy.contiguous()
        dx = torch.empty(N, H, W, C, dtype=dy.dtype, device=dy.device)
        _nat.call("pa_gap_nhwc_bwd", _nat.ptr(dy), _nat.ptr(dx), N, H * W, C, _nat.stream())
        return dx


def global_avg_pool_nhwc(x):
    return _tape.apply(_GapNHWC, x)
