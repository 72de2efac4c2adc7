"""Neural-network operators: conv / pool / norm / dropout / softmax / losses / embedding.

Parity: paddle/fluid/operators/{conv,conv_transpose,pool,pool_with_index,batch_norm,
layer_norm,lrn,dropout,softmax,cross_entropy,softmax_with_cross_entropy,
sigmoid_cross_entropy_with_logits,lookup_table,one_hot,top_k,accuracy,
hinge_loss,huber_loss,log_loss,margin_rank_loss,rank_loss,modified_huber_loss,
smooth_l1_loss,label_smooth,bilinear_interp,pad,pad2d,crop,im2sequence,spp,unpool,
roi_pool}_op.* (SURVEY §2.7).

On the HIP device, layer_norm / softmax / lookup_table go through the hand-written
gfx950 kernels (paddle_amd.ops); softmax_with_cross_entropy (Softmax + Loss in one
row pass, grad from the Softmax output) and the pointwise losses (hinge, huber,
log, modified huber, sigmoid CE; explicit grad ops) through csrc/kernels/
fluid_ops.hip (ops/fluidk.py); conv /
conv_transpose (2-D, 3-D, grouped) and pool / pool_with_index / unpool run on the
channel-first kernels of csrc/kernels/convnd.hip (ops/convnd.py).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import ops as K
from ..autograd import engine as _eager
from ..framework import core
from ..framework.op_kernel_type import LibraryType, register_op_kernel
from ..framework.registry import register_op
from ..ops import convnd as _cnd
from ..ops import fluidk as _fk
from ..ops import fused as _fused
from ..ops import oplib as _oplib

# ------------------------------------------------------------------ conv


def _conv_attrs(extra=None):
    a = {"strides": [1, 1], "paddings": [0, 0], "dilations": [1, 1], "groups": 1, "use_cudnn": True,
         "use_mkldnn": False, "data_format": "AnyLayout", "workspace_size_MB": 4096, "exhaustive_search": False}
    a.update(extra or {})
    return a


@register_op("conv2d", ["Input", "Filter", "Bias?"], ["Output"], _conv_attrs())
def conv2d(ctx):
    x, w = ctx.input("Input"), ctx.input("Filter")
    b = ctx.input("Bias") if ctx.has_input("Bias") else None
    if _cnd.supported_conv(x, w, ctx.attr("groups") or 1):
        ctx.set_output("Output", _cnd.conv_nd(x, w, b, ctx.attr("strides"), ctx.attr("paddings"),
                                              ctx.attr("dilations"), ctx.attr("groups") or 1))
        return
    y = F.conv2d(x, w.to(x.dtype), ctx.input("Bias") if ctx.has_input("Bias") else None,
                 tuple(ctx.attr("strides")), tuple(ctx.attr("paddings")), tuple(ctx.attr("dilations")),
                 ctx.attr("groups") or 1)
    ctx.set_output("Output", y)


@register_op("depthwise_conv2d", ["Input", "Filter", "Bias?"], ["Output"], _conv_attrs())
def depthwise_conv2d(ctx):
    conv2d(ctx)


@register_op("conv3d", ["Input", "Filter", "Bias?"], ["Output"],
             _conv_attrs({"strides": [1, 1, 1], "paddings": [0, 0, 0], "dilations": [1, 1, 1]}))
def conv3d(ctx):
    x, w = ctx.input("Input"), ctx.input("Filter")
    if _cnd.supported_conv(x, w, ctx.attr("groups") or 1):
        ctx.set_output("Output", _cnd.conv_nd(x, w, None, ctx.attr("strides"), ctx.attr("paddings"),
                                              ctx.attr("dilations"), ctx.attr("groups") or 1))
        return
    y = F.conv3d(x, w.to(x.dtype), None, tuple(ctx.attr("strides")), tuple(ctx.attr("paddings")),
                 tuple(ctx.attr("dilations")), ctx.attr("groups") or 1)
    ctx.set_output("Output", y)


@register_op("conv2d_grad", ["Input", "Filter", "Bias?", "Output?", "Output@GRAD"],
             ["Input@GRAD?", "Filter@GRAD?", "Bias@GRAD?"], _conv_attrs(), grad=None, no_infer=True)
def conv2d_grad(ctx):
    """Explicit data/filter gradients (no forward recompute)."""
    x, w, dy = ctx.input("Input"), ctx.input("Filter"), ctx.input("Output@GRAD")
    st, pd, dl, g = (tuple(ctx.attr("strides")), tuple(ctx.attr("paddings")), tuple(ctx.attr("dilations")),
                     ctx.attr("groups") or 1)
    if _cnd.supported_conv(x, w, g) and dy.is_cuda:
        # the HIP conv's dgrad / wgrad kernels directly (no forward recompute)
        dx, dw = _cnd.conv_grads(x.detach(), w.detach(), dy, st, pd, dl, g, ctx.has_output("Input@GRAD"),
                                 ctx.has_output("Filter@GRAD"))
        if dx is not None:
            ctx.set_output("Input@GRAD", dx)
        if dw is not None:
            ctx.set_output("Filter@GRAD", dw)
        if ctx.has_output("Bias@GRAD"):
            ctx.set_output("Bias@GRAD", _cnd._bias_grad(dy.float().contiguous()).to(dy.dtype))
        return
    if ctx.has_output("Input@GRAD"):
        ctx.set_output("Input@GRAD", torch.nn.grad.conv2d_input(x.shape, w, dy, st, pd, dl, g))
    if ctx.has_output("Filter@GRAD"):
        ctx.set_output("Filter@GRAD", torch.nn.grad.conv2d_weight(x, w.shape, dy, st, pd, dl, g))
    if ctx.has_output("Bias@GRAD"):
        ctx.set_output("Bias@GRAD", dy.sum((0, 2, 3)))


@register_op("conv2d_transpose", ["Input", "Filter"], ["Output"],
             _conv_attrs({"output_size": []}))
def conv2d_transpose(ctx):
    x, w = ctx.input("Input"), ctx.input("Filter")
    st, pd, dl = tuple(ctx.attr("strides")), tuple(ctx.attr("paddings")), tuple(ctx.attr("dilations"))
    if _cnd.supported_conv_transpose(x, w, ctx.attr("groups") or 1):
        y = _cnd.conv_transpose_nd(x, w, st, pd, dl, ctx.attr("groups") or 1)
    else:
        y = F.conv_transpose2d(x, w.to(x.dtype), None, st, pd, 0, ctx.attr("groups") or 1, dl)
    osz = ctx.attr("output_size")
    if osz:
        y = y[..., :osz[0], :osz[1]]
    ctx.set_output("Output", y)


@register_op("conv3d_transpose", ["Input", "Filter"], ["Output"],
             _conv_attrs({"strides": [1, 1, 1], "paddings": [0, 0, 0], "dilations": [1, 1, 1], "output_size": []}))
def conv3d_transpose(ctx):
    x, w = ctx.input("Input"), ctx.input("Filter")
    if _cnd.supported_conv_transpose(x, w, ctx.attr("groups") or 1):
        y = _cnd.conv_transpose_nd(x, w, ctx.attr("strides"), ctx.attr("paddings"), ctx.attr("dilations"),
                                   ctx.attr("groups") or 1)
        osz = ctx.attr("output_size")
        if osz:
            y = y[..., :osz[0], :osz[1], :osz[2]]
        ctx.set_output("Output", y)
        return
    y = F.conv_transpose3d(x, w.to(x.dtype), None, tuple(ctx.attr("strides")), tuple(ctx.attr("paddings")), 0,
                           ctx.attr("groups") or 1, tuple(ctx.attr("dilations")))
    ctx.set_output("Output", y)


# ------------------------------------------------------------------ pool


def _pool_out(size, k, s, p, ceil):
    if ceil:
        return (size - k + 2 * p + s - 1) // s + 1
    return (size - k + 2 * p) // s + 1


@register_op("pool2d", ["X"], ["Out"], {"pooling_type": "max", "ksize": [2, 2], "global_pooling": False,
                                        "strides": [1, 1], "paddings": [0, 0], "exclusive": True,
                                        "ceil_mode": False, "use_cudnn": True, "use_mkldnn": False,
                                        "data_format": "AnyLayout"})
def pool2d(ctx):
    x = ctx.input("X")
    k, s, p = list(ctx.attr("ksize")), list(ctx.attr("strides")), list(ctx.attr("paddings"))
    if ctx.attr("global_pooling"):
        k, p = [x.shape[2], x.shape[3]], [0, 0]
    if _cnd.supported_pool(x) and x.dim() == 4:
        ctx.set_output("Out", _cnd.pool_nd(x, ctx.attr("pooling_type"), k, s, p, ctx.attr("exclusive"),
                                           ctx.attr("ceil_mode")))
        return
    if ctx.attr("pooling_type") == "max":
        y = F.max_pool2d(x, k, s, p, ceil_mode=ctx.attr("ceil_mode"))
    else:
        y = F.avg_pool2d(x, k, s, p, ceil_mode=ctx.attr("ceil_mode"), count_include_pad=not ctx.attr("exclusive"))
    ctx.set_output("Out", y)


@register_op("pool3d", ["X"], ["Out"], {"pooling_type": "max", "ksize": [2, 2, 2], "global_pooling": False,
                                        "strides": [1, 1, 1], "paddings": [0, 0, 0], "exclusive": True,
                                        "ceil_mode": False, "use_cudnn": True})
def pool3d(ctx):
    x = ctx.input("X")
    k, s, p = list(ctx.attr("ksize")), list(ctx.attr("strides")), list(ctx.attr("paddings"))
    if ctx.attr("global_pooling"):
        k, p = list(x.shape[2:]), [0, 0, 0]
    if _cnd.supported_pool(x) and x.dim() == 5:
        ctx.set_output("Out", _cnd.pool_nd(x, ctx.attr("pooling_type"), k, s, p, ctx.attr("exclusive"),
                                           ctx.attr("ceil_mode")))
        return
    if ctx.attr("pooling_type") == "max":
        y = F.max_pool3d(x, k, s, p, ceil_mode=ctx.attr("ceil_mode"))
    else:
        y = F.avg_pool3d(x, k, s, p, ceil_mode=ctx.attr("ceil_mode"), count_include_pad=not ctx.attr("exclusive"))
    ctx.set_output("Out", y)


@register_op("max_pool2d_with_index", ["X"], ["Out", "Mask"], {"ksize": [2, 2], "global_pooling": False,
                                                               "strides": [1, 1], "paddings": [0, 0]})
def max_pool2d_with_index(ctx):
    x = ctx.input("X")
    k, s, p = ctx.attr("ksize"), ctx.attr("strides"), ctx.attr("paddings")
    if ctx.attr("global_pooling"):
        k, p = [x.shape[2], x.shape[3]], [0, 0]
    if _cnd.supported_pool(x) and x.dim() == 4:
        y, idx = _cnd.pool_nd(x, "max", k, s, p, return_mask=True)
        ctx.set_output("Out", y)
        ctx.set_output("Mask", idx)
        return
    y, idx = F.max_pool2d(x, k, s, p, return_indices=True)
    ctx.set_output("Out", y)
    ctx.set_output("Mask", idx.to(torch.int32))


@register_op("unpool", ["X", "Indices"], ["Out"], {"unpooling_type": "max", "ksize": [2, 2], "strides": [2, 2],
                                                   "paddings": [0, 0]})
def unpool(ctx):
    x, idx = ctx.input("X"), ctx.input("Indices").long()
    k, s, p = ctx.attr("ksize"), ctx.attr("strides"), ctx.attr("paddings")
    if _cnd.supported_pool(x) and x.dim() == 4:
        ctx.set_output("Out", _cnd.unpool2d(x, idx, k, s, p))
        return
    ctx.set_output("Out", F.max_unpool2d(x, idx, k, s, p))


@register_op("spp", ["X"], ["Out"], {"pyramid_height": 1, "pooling_type": "max"})
def spp(ctx):
    x = ctx.input("X")
    N, C, H, W = x.shape
    outs = []
    for lvl in range(ctx.attr("pyramid_height")):
        # spp_op.h: kernel = ceil(size / bins), stride = kernel, padding =
        # (kernel * bins - size + 1) / 2; avg pooling counts valid elements only
        bins = 2 ** lvl
        kh, kw = -(-H // bins), -(-W // bins)
        ph, pw = (kh * bins - H + 1) // 2, (kw * bins - W + 1) // 2
        pad = (pw, kw * bins - W - pw, ph, kh * bins - H - ph)
        if _cnd.supported_pool(x) and kh * bins - H - ph <= ph and kw * bins - W - pw <= pw:
            # the native NCHW pool kernel: symmetric padding (the right/bottom pad is
            # never larger, and floor() drops the partial window it would add), max
            # over valid pixels / exclusive average -- spp_op.h's semantics
            o = _cnd.pool_nd(x, ctx.attr("pooling_type"), (kh, kw), (kh, kw), (ph, pw), exclusive=True)
            outs.append(o.reshape(N, -1))
            continue
        if ctx.attr("pooling_type") == "max":
            o = F.max_pool2d(F.pad(x, pad, value=float("-inf")), (kh, kw), (kh, kw))
        else:
            ones = F.pad(torch.ones(1, 1, H, W, dtype=x.dtype, device=x.device), pad)
            o = F.avg_pool2d(F.pad(x, pad), (kh, kw), (kh, kw)) / F.avg_pool2d(ones, (kh, kw), (kh, kw))
        outs.append(o.reshape(N, -1))
    ctx.set_output("Out", torch.cat(outs, 1))


# ------------------------------------------------------------------ normalisation


@register_op("batch_norm", ["X", "Scale", "Bias", "Mean", "Variance"],
             ["Y", "MeanOut", "VarianceOut", "SavedMean~", "SavedVariance~"],
             {"momentum": 0.9, "epsilon": 1e-5, "is_test": False, "data_layout": "NCHW", "use_mkldnn": False,
              "fuse_with_relu": False, "use_global_stats": False})
def batch_norm(ctx):
    x = ctx.input("X")
    sc, b, m, v = ctx.input("Scale"), ctx.input("Bias"), ctx.input("Mean"), ctx.input("Variance")
    eps, mom = ctx.attr("epsilon"), ctx.attr("momentum")
    nhwc = ctx.attr("data_layout") == "NHWC"
    xc = x.movedim(-1, 1) if nhwc and x.dim() > 2 else x
    test = ctx.attr("is_test") or ctx.attr("use_global_stats")
    if _cnd.supported_bn(xc.contiguous()) and sc is not None and b is not None:
        y, mean_out, var_out, saved_m, saved_v = _cnd.batch_norm_nchw(
            xc.contiguous(), sc, b, m, v, mom, eps, training=not test, relu=bool(ctx.attr("fuse_with_relu")))
        if nhwc and x.dim() > 2:
            y = y.movedim(1, -1)
        ctx.set_output("Y", y)
        ctx.set_output("MeanOut", mean_out.to(m.dtype))
        ctx.set_output("VarianceOut", var_out.to(v.dtype))
        ctx.set_output("SavedMean", saved_m)
        ctx.set_output("SavedVariance", saved_v)
        return
    if test:
        y = F.batch_norm(xc, m, v, sc, b, False, 0.0, eps)
        mean_out, var_out = m, v
        saved_m, saved_v = m, v
    else:
        dims = [0] + list(range(2, xc.dim()))
        xf = xc.float()
        bm = xf.mean(dims)
        bv = xf.var(dims, unbiased=False)
        shape = [1, -1] + [1] * (xc.dim() - 2)
        y = ((xf - bm.reshape(shape)) * torch.rsqrt(bv.reshape(shape) + eps) * sc.float().reshape(shape)
             + b.float().reshape(shape)).to(x.dtype)
        mean_out = (m * mom + bm.detach() * (1 - mom)).to(m.dtype)
        var_out = (v * mom + bv.detach() * (1 - mom)).to(v.dtype)
        saved_m, saved_v = bm, torch.rsqrt(bv + eps)
    if ctx.attr("fuse_with_relu"):
        y = F.relu(y)
    if nhwc and x.dim() > 2:
        y = y.movedim(1, -1)
    ctx.set_output("Y", y)
    ctx.set_output("MeanOut", mean_out.detach() if not test else mean_out)
    ctx.set_output("VarianceOut", var_out.detach() if not test else var_out)
    ctx.set_output("SavedMean", saved_m)
    ctx.set_output("SavedVariance", saved_v)


@register_op("layer_norm", ["X", "Scale?", "Bias?"], ["Y", "Mean~", "Variance~"],
             {"epsilon": 1e-5, "begin_norm_axis": 1, "is_test": False})
def layer_norm(ctx):
    x = ctx.input("X")
    ax = ctx.attr("begin_norm_axis")
    lead = x.shape[:ax]
    x2 = x.reshape(int(torch.tensor(lead).prod()) if lead else 1, -1)
    sc = ctx.input("Scale") if ctx.has_input("Scale") else None
    b = ctx.input("Bias") if ctx.has_input("Bias") else None
    eps = ctx.attr("epsilon")
    sc1 = sc.reshape(-1) if sc is not None else None
    b1 = b.reshape(-1).to(x2.dtype) if b is not None else None
    if not ctx.meta and _fused.norm_kernel_ok(x2, sc1):
        # one HIP pass: Y plus the row statistics the grad op reads back
        y, mean, rstd = _fused.layer_norm_stats(x2, sc1, b1, eps)
        ctx.set_output("Y", y.reshape(x.shape))
        ctx.set_output("Mean", mean)
        ctx.set_output("Variance", rstd.pow(-2) - eps)
        return
    y = K.layer_norm(x2, sc1, b1, eps)
    xf = x2.float()
    ctx.set_output("Y", y.reshape(x.shape))
    ctx.set_output("Mean", xf.mean(1))
    ctx.set_output("Variance", xf.var(1, unbiased=False))


@register_op("layer_norm_grad", ["X", "Scale?", "Bias?", "Mean", "Variance", "Y?", "Y@GRAD"],
             ["X@GRAD", "Scale@GRAD?", "Bias@GRAD?"], {"epsilon": 1e-5, "begin_norm_axis": 1, "is_test": False},
             grad=None, no_infer=True)
def layer_norm_grad(ctx):
    """Explicit layer_norm grad from the saved Mean / Variance (layer_norm_op.h
    LayerNormGradKernel): the norm kernel's backward on the device, the same closed
    form in torch on the host."""
    x, dy = ctx.input("X"), ctx.input("Y@GRAD")
    ax = ctx.attr("begin_norm_axis")
    eps = ctx.attr("epsilon")
    rows = 1
    for d in x.shape[:ax]:
        rows *= int(d)
    x2, dy2 = x.reshape(rows, -1), dy.reshape(rows, -1).to(x.dtype)
    sc = ctx.input("Scale").reshape(-1) if ctx.has_input("Scale") else None
    has_b = ctx.has_input("Bias")
    mean = ctx.input("Mean").reshape(-1).float()
    rstd = torch.rsqrt(ctx.input("Variance").reshape(-1).float() + eps)
    if _fused.norm_kernel_ok(x2, sc):
        dx, dw, db = _fused.layer_norm_stats_grad(dy2, x2, sc, mean, rstd, has_b)
    else:
        xh = (x2.float() - mean[:, None]) * rstd[:, None]
        g = dy2.float()
        dw = (g * xh).sum(0) if sc is not None else None
        db = g.sum(0) if has_b else None
        gx = g * sc.float()[None, :] if sc is not None else g
        dx = rstd[:, None] * (gx - gx.mean(1, keepdim=True) - xh * (gx * xh).mean(1, keepdim=True))
        dx = dx.to(x.dtype)
    ctx.set_output("X@GRAD", dx.reshape(x.shape))
    if ctx.has_output("Scale@GRAD") and sc is not None:
        ctx.set_output("Scale@GRAD", dw.to(sc.dtype).reshape(ctx.input("Scale").shape))
    if ctx.has_output("Bias@GRAD") and has_b:
        ctx.set_output("Bias@GRAD", db.to(ctx.input("Bias").dtype).reshape(ctx.input("Bias").shape))


@register_op("lrn", ["X"], ["Out", "MidOut~"], {"n": 5, "k": 2.0, "alpha": 1e-4, "beta": 0.75})
def lrn(ctx):
    x = ctx.input("X")
    n, k, a, b = ctx.attr("n"), ctx.attr("k"), ctx.attr("alpha"), ctx.attr("beta")
    r = _oplib.lrn_op(x, n, k, a, b) if x.is_cuda else None
    if r is not None:
        ctx.set_output("Out", r[0])
        ctx.set_output("MidOut", r[1])
        return
    sq = (x * x).unsqueeze(1)
    # window [c - (n-1)//2, c - (n-1)//2 + n) (lrn_op.cc: start = -(n - 1) / 2)
    pad = F.pad(sq, (0, 0, 0, 0, (n - 1) // 2, n // 2))
    s = F.avg_pool3d(pad, (n, 1, 1), stride=1).squeeze(1) * n
    mid = k + a * s
    ctx.set_output("Out", x / mid.pow(b))
    ctx.set_output("MidOut", mid)


@register_op("dropout", ["X"], ["Out", "Mask~"], {"dropout_prob": 0.5, "is_test": False, "fix_seed": False,
                                                  "seed": 0, "dropout_implementation": "downgrade_in_infer"})
def dropout(ctx):
    x = ctx.input("X")
    p = ctx.attr("dropout_prob")
    upscale = ctx.attr("dropout_implementation") == "upscale_in_train"
    if ctx.attr("is_test"):
        ctx.set_output("Out", x if upscale else x * (1.0 - p))
        return
    if x.is_cuda and not ctx.meta:
        # Philox4x32-10 counter RNG kernel (dropout_op.cu:27 uses curand); uint8 mask
        r = _oplib.dropout_op(x, p, int(ctx.attr("seed")) if ctx.attr("fix_seed") else None, upscale)
        if r is not None:
            ctx.set_output("Out", r[0])
            ctx.set_output("Mask", r[1])
            return
    g = None
    if ctx.attr("fix_seed") and not ctx.meta:
        g = torch.Generator(device=x.device)
        g.manual_seed(int(ctx.attr("seed")))
    mask = (torch.rand(x.shape, device=x.device, generator=g) >= p).to(x.dtype) if not ctx.meta \
        else torch.empty_like(x)
    out = x * mask / (1.0 - p) if (upscale and p < 1.0) else x * mask
    ctx.set_output("Out", out)
    ctx.set_output("Mask", mask)


@register_op("dropout_grad", ["Mask", "Out@GRAD", "X?", "Out?"], ["X@GRAD"],
             {"dropout_prob": 0.5, "is_test": False, "fix_seed": False, "seed": 0,
              "dropout_implementation": "downgrade_in_infer"}, grad=None, no_infer=True)
def dropout_grad(ctx):
    m, d = ctx.input("Mask"), ctx.input("Out@GRAD")
    p = ctx.attr("dropout_prob")
    if m.dtype == torch.uint8:  # native Philox mask
        sc = 1.0 / (1.0 - p) if (ctx.attr("dropout_implementation") == "upscale_in_train" and p < 1.0) else 1.0
        g = _oplib.mask_mul(d, m, sc)
        ctx.set_output("X@GRAD", g if g is not None else d * m.to(d.dtype) * sc)
        return
    g = d * m
    if ctx.attr("dropout_implementation") == "upscale_in_train" and p < 1.0:
        g = g / (1.0 - p)
    ctx.set_output("X@GRAD", g)


def _dropout_grad_maker(op, no_grad):
    return [dict(type="dropout_grad", inputs={"Mask": op.output("Mask"), "Out@GRAD": [op.output("Out")[0] + "@GRAD"]},
                 outputs={"X@GRAD": [op.input("X")[0] + "@GRAD"]}, attrs=dict(op.all_attrs()))]


from ..framework.registry import OP_REGISTRY as _REG  # noqa: E402

_REG["dropout"].grad_maker = _dropout_grad_maker

# ------------------------------------------------------------------ softmax & losses


@register_op("softmax", ["X"], ["Out"], {"use_cudnn": False, "use_mkldnn": False, "axis": -1,
                                         "data_format": "AnyLayout", "is_test": False})
def softmax(ctx):
    x = ctx.input("X")
    ctx.set_output("Out", K.softmax(x, ctx.attr("axis")))


@register_op("log_softmax", ["X"], ["Out"], {"axis": -1})
def log_softmax(ctx):
    ctx.set_output("Out", K.softmax(ctx.input("X"), ctx.attr("axis"), log=True))


def _gather_label(p, label):
    return p.gather(-1, label.long().reshape(p.shape[:-1] + (1,)))


@register_op("cross_entropy", ["X", "Label"], ["Y"], {"soft_label": False, "ignore_index": -100})
def cross_entropy(ctx):
    """-log(X[label]) with X a probability distribution (cross_entropy_op.h)."""
    x, lab = ctx.input("X"), ctx.input("Label")
    from ..ops import nnmisc as _nm
    r = _nm.cross_entropy(x, lab, ctx.attr("soft_label"), ctx.attr("ignore_index"))
    if r is not None:  # math/cross_entropy.cu counterpart (nnmisc.hip)
        ctx.set_output("Y", r)
        return
    if ctx.attr("soft_label"):
        y = -(lab * torch.log(x)).sum(-1, keepdim=True)
    else:
        lab2 = lab.long().reshape(x.shape[:-1] + (1,))
        ign = lab2 == ctx.attr("ignore_index")
        picked = x.gather(-1, torch.where(ign, torch.zeros_like(lab2), lab2))
        y = torch.where(ign, torch.zeros_like(picked), -torch.log(picked))
    ctx.set_output("Y", y)


@register_op("softmax_with_cross_entropy", ["Logits", "Label"], ["Softmax", "Loss"],
             {"soft_label": False, "ignore_index": -100, "numeric_stable_mode": True, "axis": -1})
def softmax_with_cross_entropy(ctx):
    x, lab = ctx.input("Logits"), ctx.input("Label")
    if _fk.ok(x) and not ctx.meta and ctx.attr("axis") in (-1, x.dim() - 1):
        # one HIP block per row: online max / sum, then probabilities + row loss
        soft = ctx.attr("soft_label")
        prob, loss = _fk.softmax_ce(x, None if soft else lab, lab if soft else None, ctx.attr("ignore_index"))
        ctx.set_output("Softmax", prob)
        ctx.set_output("Loss", loss)
        return
    logp = torch.log_softmax(x.float(), -1)
    if ctx.attr("soft_label"):
        loss = -(lab.float() * logp).sum(-1, keepdim=True)
    else:
        lab2 = lab.long().reshape(x.shape[:-1] + (1,))
        ign = lab2 == ctx.attr("ignore_index")
        picked = logp.gather(-1, torch.where(ign, torch.zeros_like(lab2), lab2))
        loss = torch.where(ign, torch.zeros_like(picked), -picked)
    ctx.set_output("Softmax", torch.exp(logp).to(x.dtype))
    ctx.set_output("Loss", loss.to(x.dtype))


@register_op("softmax_with_cross_entropy_grad", ["Label", "Softmax", "Loss@GRAD", "Logits?", "Loss?"],
             ["Logits@GRAD"], {"soft_label": False, "ignore_index": -100, "numeric_stable_mode": True, "axis": -1},
             grad=None, no_infer=True)
def softmax_with_cross_entropy_grad(ctx):
    p, lab, d = ctx.input("Softmax"), ctx.input("Label"), ctx.input("Loss@GRAD")
    if _fk.ok(p, d) and not ctx.meta and ctx.attr("axis") in (-1, p.dim() - 1):
        soft = ctx.attr("soft_label")
        ctx.set_output("Logits@GRAD", _fk.softmax_ce_grad(p, d, None if soft else lab, lab if soft else None,
                                                          ctx.attr("ignore_index")))
        return
    if ctx.attr("soft_label"):
        g = (p - lab.to(p.dtype)) * d
    else:
        lab2 = lab.long().reshape(p.shape[:-1] + (1,))
        ign = lab2 == ctx.attr("ignore_index")
        oh = torch.zeros_like(p).scatter_(-1, torch.where(ign, torch.zeros_like(lab2), lab2), 1.0)
        g = (p - oh) * d * (~ign).to(p.dtype)
    ctx.set_output("Logits@GRAD", g)


def _swce_grad_maker(op, no_grad):
    return [dict(type="softmax_with_cross_entropy_grad",
                 inputs={"Label": op.input("Label"), "Softmax": op.output("Softmax"),
                         "Loss@GRAD": [op.output("Loss")[0] + "@GRAD"]},
                 outputs={"Logits@GRAD": [op.input("Logits")[0] + "@GRAD"]}, attrs=dict(op.all_attrs()))]


_REG["softmax_with_cross_entropy"].grad_maker = _swce_grad_maker


@register_op("sigmoid_cross_entropy_with_logits", ["X", "Label"], ["Out"], {"ignore_index": -100})
def sigmoid_ce(ctx):
    x, lab = ctx.input("X"), ctx.input("Label")
    if _fk.ok(x) and not ctx.meta:
        out = _fk.loss_fwd("sigmoid_cross_entropy_with_logits", x, lab)[0]
    else:
        out = F.binary_cross_entropy_with_logits(x, lab.to(x.dtype), reduction="none")
    out = torch.where(lab == ctx.attr("ignore_index"), torch.zeros_like(out), out)
    ctx.set_output("Out", out)


@register_op("sigmoid_cross_entropy_with_logits_grad", ["X", "Label", "Out?", "Out@GRAD"], ["X@GRAD", "Label@GRAD?"],
             {"ignore_index": -100}, grad=None, no_infer=True)
def sigmoid_ce_grad(ctx):
    x, lab, g = ctx.input("X"), ctx.input("Label"), ctx.input("Out@GRAD")
    if _fk.ok(x, g) and not ctx.meta:
        gx = _fk.loss_bwd("sigmoid_cross_entropy_with_logits", x, lab, g)
    else:
        gx = g * (torch.sigmoid(x) - lab.to(x.dtype))
    ctx.set_output("X@GRAD", torch.where(lab == ctx.attr("ignore_index"), torch.zeros_like(gx), gx))


@register_op("bpr_loss", ["X", "Label"], ["Y"], {})
def bpr_loss(ctx):
    x, lab = ctx.input("X"), ctx.input("Label").long().reshape(-1)
    pos = x.gather(1, lab[:, None])
    diff = pos - x
    y = -F.logsigmoid(diff)
    mask = torch.ones_like(x).scatter_(1, lab[:, None], 0.0)
    ctx.set_output("Y", (y * mask).sum(1, keepdim=True) / max(1, x.shape[1] - 1))


@register_op("hinge_loss", ["Logits", "Labels"], ["Loss"], {})
def hinge_loss(ctx):
    x, y = ctx.input("Logits"), ctx.input("Labels")
    if _fk.ok(x) and not ctx.meta:
        ctx.set_output("Loss", _fk.loss_fwd("hinge_loss", x, y)[0])
        return
    ctx.set_output("Loss", F.relu(1 - x * (2 * y - 1)))


@register_op("hinge_loss_grad", ["Logits", "Labels", "Loss?", "Loss@GRAD"], ["Logits@GRAD", "Labels@GRAD?"], {},
             grad=None, no_infer=True)
def hinge_loss_grad(ctx):
    x, y, g = ctx.input("Logits"), ctx.input("Labels"), ctx.input("Loss@GRAD")
    if _fk.ok(x, g) and not ctx.meta:
        ctx.set_output("Logits@GRAD", _fk.loss_bwd("hinge_loss", x, y, g))
        return
    s = 2 * y.to(x.dtype) - 1
    ctx.set_output("Logits@GRAD", g * torch.where(x * s < 1, -s, torch.zeros_like(s)))


@register_op("huber_loss", ["X", "Y"], ["Residual~", "Out"], {"delta": 1.0})
def huber_loss(ctx):
    x, y = ctx.input("X"), ctx.input("Y")
    if _fk.ok(x) and not ctx.meta:
        out, res = _fk.loss_fwd("huber_loss", x, y, ctx.attr("delta"), want_res=True)
        ctx.set_output("Residual", res)
        ctx.set_output("Out", out)
        return
    r = y - x
    d = ctx.attr("delta")
    a = r.abs()
    ctx.set_output("Residual", r)
    ctx.set_output("Out", torch.where(a <= d, 0.5 * r * r, d * (a - 0.5 * d)))


@register_op("huber_loss_grad", ["X", "Y", "Residual", "Out?", "Out@GRAD"], ["X@GRAD", "Y@GRAD?"], {"delta": 1.0},
             grad=None, no_infer=True)
def huber_loss_grad(ctx):
    x, y, r, g = ctx.input("X"), ctx.input("Y"), ctx.input("Residual"), ctx.input("Out@GRAD")
    d = ctx.attr("delta")
    if _fk.ok(x, g) and not ctx.meta:
        gx = _fk.loss_bwd("huber_loss", x, y, g, res=r, a=d)
    else:
        gx = g * torch.where(r.abs() <= d, -r, torch.where(r > 0, torch.full_like(r, -d), torch.full_like(r, d)))
    ctx.set_output("X@GRAD", gx)
    if ctx.has_output("Y@GRAD"):
        ctx.set_output("Y@GRAD", -gx)


@register_op("log_loss", ["Predicted", "Labels"], ["Loss"], {"epsilon": 1e-4})
def log_loss(ctx):
    p, y = ctx.input("Predicted"), ctx.input("Labels")
    e = ctx.attr("epsilon")
    if _fk.ok(p) and not ctx.meta:
        ctx.set_output("Loss", _fk.loss_fwd("log_loss", p, y, e)[0])
        return
    ctx.set_output("Loss", -y * torch.log(p + e) - (1 - y) * torch.log(1 - p + e))


@register_op("log_loss_grad", ["Predicted", "Labels", "Loss?", "Loss@GRAD"], ["Predicted@GRAD", "Labels@GRAD?"],
             {"epsilon": 1e-4}, grad=None, no_infer=True)
def log_loss_grad(ctx):
    p, y, g = ctx.input("Predicted"), ctx.input("Labels"), ctx.input("Loss@GRAD")
    e = ctx.attr("epsilon")
    if _fk.ok(p, g) and not ctx.meta:
        ctx.set_output("Predicted@GRAD", _fk.loss_bwd("log_loss", p, y, g, a=e))
        return
    y = y.to(p.dtype)
    ctx.set_output("Predicted@GRAD", g * (-y / (p + e) + (1 - y) / (1 - p + e)))


@register_op("margin_rank_loss", ["X1", "X2", "Label"], ["Out", "Activated~"], {"margin": 0.0})
def margin_rank_loss(ctx):
    x1, x2, lab = ctx.input("X1"), ctx.input("X2"), ctx.input("Label")
    v = -lab * (x1 - x2) + ctx.attr("margin")
    ctx.set_output("Out", F.relu(v))
    ctx.set_output("Activated", (v > 0).to(x1.dtype))


@register_op("rank_loss", ["Label", "Left", "Right"], ["Out"], {})
def rank_loss(ctx):
    lab, l, r = ctx.input("Label"), ctx.input("Left"), ctx.input("Right")
    o = l - r
    ctx.set_output("Out", torch.log1p(torch.exp(o)) - lab * o)


@register_op("modified_huber_loss", ["X", "Y"], ["IntermediateVal~", "Out"], {})
def modified_huber_loss(ctx):
    x, y = ctx.input("X"), ctx.input("Y")
    if _fk.ok(x) and not ctx.meta:
        out, z = _fk.loss_fwd("modified_huber_loss", x, y, want_res=True)
        ctx.set_output("IntermediateVal", z)
        ctx.set_output("Out", out)
        return
    z = x * (2 * y - 1)
    ctx.set_output("IntermediateVal", z)
    ctx.set_output("Out", torch.where(z < -1, -4 * z, torch.where(z < 1, (1 - z) ** 2, torch.zeros_like(z))))


@register_op("modified_huber_loss_grad", ["X", "Y", "IntermediateVal", "Out?", "Out@GRAD"], ["X@GRAD", "Y@GRAD?"],
             {}, grad=None, no_infer=True)
def modified_huber_loss_grad(ctx):
    x, y, z, g = ctx.input("X"), ctx.input("Y"), ctx.input("IntermediateVal"), ctx.input("Out@GRAD")
    if _fk.ok(x, g) and not ctx.meta:
        ctx.set_output("X@GRAD", _fk.loss_bwd("modified_huber_loss", x, y, g, res=z))
        return
    s = 2 * y.to(x.dtype) - 1
    ctx.set_output("X@GRAD", g * torch.where(z < -1, -4 * s, torch.where(z < 1, -2 * (1 - z) * s,
                                                                          torch.zeros_like(z))))


@register_op("smooth_l1_loss", ["X", "Y", "InsideWeight?", "OutsideWeight?"], ["Diff~", "Out"], {"sigma": 1.0})
def smooth_l1_loss(ctx):
    x, y = ctx.input("X"), ctx.input("Y")
    s2 = ctx.attr("sigma") ** 2
    d = x - y
    if ctx.has_input("InsideWeight"):
        d = d * ctx.input("InsideWeight")
    a = d.abs()
    v = torch.where(a < 1.0 / s2, 0.5 * d * d * s2, a - 0.5 / s2)
    if ctx.has_input("OutsideWeight"):
        v = v * ctx.input("OutsideWeight")
    ctx.set_output("Diff", d)
    ctx.set_output("Out", v.reshape(v.shape[0], -1).sum(1, keepdim=True))


@register_op("kldiv_loss", ["X", "Target"], ["Loss"], {"reduction": "mean"})
def kldiv_loss(ctx):
    x, t = ctx.input("X"), ctx.input("Target")
    l = torch.where(t > 0, t * (torch.log(t.clamp_min(1e-30)) - x), torch.zeros_like(x))
    red = ctx.attr("reduction")
    if red == "mean":
        l = l.mean().reshape(1)
    elif red == "sum":
        l = l.sum().reshape(1)
    elif red == "batchmean":
        l = (l.sum() / x.shape[0]).reshape(1)
    ctx.set_output("Loss", l)


@register_op("label_smooth", ["X", "PriorDist?"], ["Out"], {"epsilon": 0.0})
def label_smooth(ctx):
    x = ctx.input("X")
    e = ctx.attr("epsilon")
    if ctx.has_input("PriorDist"):
        ctx.set_output("Out", (1 - e) * x + e * ctx.input("PriorDist"))
    else:
        ctx.set_output("Out", (1 - e) * x + e / x.shape[-1])


# ------------------------------------------------------------------ embedding / one_hot


@register_op("lookup_table", ["W", "Ids"], ["Out"], {"is_sparse": False, "is_distributed": False,
                                                     "padding_idx": -1, "remote_prefetch": False})
def lookup_table(ctx):
    w, ids = ctx.input("W"), ctx.input("Ids")
    pad = ctx.attr("padding_idx")
    flat = ids.reshape(-1).long()
    out = K.embedding(flat, w, None if pad == -1 else pad) if not ctx.meta else torch.empty(
        flat.shape[0], w.shape[1], dtype=w.dtype, device="meta")
    shape = tuple(ids.shape[:-1]) + (w.shape[1],) if ids.dim() > 1 and ids.shape[-1] == 1 else \
        tuple(ids.shape) + (w.shape[1],)
    ctx.set_output("Out", out.reshape(shape))


@register_op("lookup_table_grad", ["W", "Ids", "Out@GRAD", "Out?"], ["W@GRAD"],
             {"is_sparse": False, "is_distributed": False, "padding_idx": -1, "remote_prefetch": False},
             grad=None, no_infer=True)
def lookup_table_grad(ctx):
    """Dense grad (scatter-add), or SelectedRows grad when is_sparse (lookup_table_op.cu:166)."""
    w, ids, d = ctx.input("W"), ctx.input("Ids"), ctx.input("Out@GRAD")
    flat = ids.reshape(-1).long()
    d2 = d.reshape(flat.shape[0], -1)
    pad = ctx.attr("padding_idx")
    if pad != -1:
        d2 = d2 * (flat != pad).to(d2.dtype)[:, None]
    if ctx.attr("is_sparse"):
        ctx.set_output("W@GRAD", core.SelectedRows(flat.tolist(), w.shape[0], d2))
    else:
        g = torch.zeros(w.shape, dtype=torch.float32, device=w.device)
        g.index_add_(0, flat, d2.float())
        ctx.set_output("W@GRAD", g.to(w.dtype))


def _lt_grad_maker(op, no_grad):
    return [dict(type="lookup_table_grad", inputs={"W": op.input("W"), "Ids": op.input("Ids"),
                                                    "Out@GRAD": [op.output("Out")[0] + "@GRAD"]},
                 outputs={"W@GRAD": [op.input("W")[0] + "@GRAD"]}, attrs=dict(op.all_attrs()))]


_REG["lookup_table"].grad_maker = _lt_grad_maker


@register_op("one_hot", ["X"], ["Out"], {"depth": 1, "dtype": 5})
def one_hot(ctx):
    x = ctx.input("X").long()
    d = ctx.attr("depth")
    if x.is_cuda and not ctx.meta:
        xs = x.reshape(x.shape[:-1] if x.dim() > 1 and x.shape[-1] == 1 else x.shape)
        r = _oplib.one_hot(xs, d)
        if r is not None:
            ctx.set_output("Out", r.to(core.to_torch_dtype(ctx.attr("dtype"))))
            return
    out = F.one_hot(x.reshape(x.shape[:-1] if x.dim() > 1 and x.shape[-1] == 1 else x.shape), d) if not ctx.meta \
        else torch.empty(tuple(x.shape[:-1]) + (d,), device="meta")
    ctx.set_output("Out", out.to(core.to_torch_dtype(ctx.attr("dtype"))))


# ------------------------------------------------------------------ top-k / accuracy


@register_op("top_k", ["X"], ["Out", "Indices"], {"k": 1})
def top_k(ctx):
    x = ctx.input("X")
    r = _oplib.topk_op(x, ctx.attr("k")) if x.is_cuda else None
    v, i = r if r is not None else torch.topk(x, ctx.attr("k"), -1)
    ctx.set_output("Out", v)
    ctx.set_output("Indices", i)


@register_op("accuracy", ["Out", "Indices", "Label"], ["Accuracy", "Correct", "Total"], {}, grad=None)
def accuracy(ctx):
    idx, lab = ctx.input("Indices"), ctx.input("Label")
    r = _oplib.accuracy_op(idx, lab) if idx.is_cuda else None
    if r is not None:
        ctx.set_output("Accuracy", r[0])
        ctx.set_output("Correct", r[1])
        ctx.set_output("Total", r[2])
        return
    lab = lab.reshape(-1, 1).to(idx.dtype)
    correct = (idx == lab).any(1).sum()
    total = torch.tensor(idx.shape[0], device=idx.device)
    ctx.set_output("Accuracy", (correct.float() / max(1, idx.shape[0])).reshape(1))
    ctx.set_output("Correct", correct.reshape(1).to(torch.int32))
    ctx.set_output("Total", total.reshape(1).to(torch.int32))


# ------------------------------------------------------------------ interp / pad / crop


@register_op("bilinear_interp", ["X", "OutSize?"], ["Out"], {"out_h": -1, "out_w": -1, "scale": 0.0,
                                                             "interp_method": "bilinear", "align_corners": True})
def bilinear_interp(ctx):
    x = ctx.input("X")
    if ctx.has_input("OutSize"):
        oh, ow = [int(v) for v in ctx.input("OutSize").reshape(-1).tolist()]
    else:
        oh, ow = ctx.attr("out_h"), ctx.attr("out_w")
        if (oh <= 0 or ow <= 0) and ctx.attr("scale") > 0:
            oh, ow = int(x.shape[2] * ctx.attr("scale")), int(x.shape[3] * ctx.attr("scale"))
    mode = "bilinear" if ctx.attr("interp_method") == "bilinear" else "nearest"
    from ..ops import nnmisc as _nm
    r = _nm.interpolate(x, oh, ow, mode, ctx.attr("align_corners"))
    if r is not None:  # interpolation kernels (nnmisc.hip)
        ctx.set_output("Out", r)
        return
    kw = {"align_corners": ctx.attr("align_corners")} if mode == "bilinear" else {}
    ctx.set_output("Out", F.interpolate(x, (oh, ow), mode=mode, **kw))


register_op("nearest_interp", ["X", "OutSize?"], ["Out"], {"out_h": -1, "out_w": -1, "scale": 0.0,
                                                           "interp_method": "nearest", "align_corners": True})(
    bilinear_interp)


@register_op("pad", ["X"], ["Out"], {"paddings": [], "pad_value": 0.0})
def pad(ctx):
    x = ctx.input("X")
    p = ctx.attr("paddings")
    tp = []
    for i in reversed(range(x.dim())):
        tp += [p[2 * i], p[2 * i + 1]]
    ctx.set_output("Out", F.pad(x, tp, value=ctx.attr("pad_value")))


@register_op("pad2d", ["X"], ["Out"], {"paddings": [0, 0, 0, 0], "mode": "constant", "pad_value": 0.0,
                                       "data_format": "NCHW"})
def pad2d(ctx):
    x = ctx.input("X")
    t, b, l, r = ctx.attr("paddings")
    mode = {"constant": "constant", "reflect": "reflect", "edge": "replicate"}[ctx.attr("mode")]
    nhwc = ctx.attr("data_format") == "NHWC"
    res = _oplib.pad2d_op(x, (t, b, l, r), ctx.attr("mode"), ctx.attr("pad_value"), nhwc) if x.is_cuda else None
    if res is not None:
        ctx.set_output("Out", res)
        return
    xc = x.permute(0, 3, 1, 2) if nhwc else x
    kw = {"value": ctx.attr("pad_value")} if mode == "constant" else {}
    y = F.pad(xc, (l, r, t, b), mode=mode, **kw)
    ctx.set_output("Out", y.permute(0, 2, 3, 1) if nhwc else y)


@register_op("pad_constant_like", ["X", "Y"], ["Out"], {"pad_value": 0.0})
def pad_constant_like(ctx):
    x, y = ctx.input("X"), ctx.input("Y")
    tp = []
    for i in reversed(range(x.dim())):
        tp += [0, x.shape[i] - y.shape[i]]
    ctx.set_output("Out", F.pad(y, tp, value=ctx.attr("pad_value")))


@register_op("crop", ["X", "Y?"], ["Out"], {"offsets": [], "shape": []})
def crop(ctx):
    x = ctx.input("X")
    shape = list(ctx.input("Y").shape) if ctx.has_input("Y") else list(ctx.attr("shape"))
    off = ctx.attr("offsets") or [0] * x.dim()
    sl = tuple(slice(o, o + s) for o, s in zip(off, shape))
    ctx.set_output("Out", x[sl])


@register_op("im2sequence", ["X"], ["Out"], {"kernels": [1, 1], "strides": [1, 1], "paddings": [0, 0, 0, 0]})
def im2sequence(ctx):
    x = ctx.input("X")
    kh, kw = ctx.attr("kernels")
    pt, pl, pb, pr = ctx.attr("paddings")
    xp = F.pad(x, (pl, pr, pt, pb))
    cols = F.unfold(xp, (kh, kw), stride=tuple(ctx.attr("strides")))  # N, C*kh*kw, L
    N, CK, L = cols.shape
    out = cols.transpose(1, 2).reshape(N * L, CK)
    ctx.set_output("Out", out, [list(range(0, N * L + 1, L))])


def _roi_batch_ids(ctx, rois):
    lod = ctx.input_lod("ROIs")
    if not lod:
        return [0] * rois.shape[0]
    off, ids = lod[0], []
    for b in range(len(off) - 1):
        ids += [b] * (off[b + 1] - off[b])
    return ids


@register_op("roi_pool", ["X", "ROIs"], ["Out", "Argmax~"], {"spatial_scale": 1.0, "pooled_height": 1,
                                                             "pooled_width": 1})
def roi_pool(ctx):
    """Max pooling over ROI bins (roi_pool_op.cu): the ROI corners are rounded half
    away from zero after scaling, bins are floor/ceil of ph * roi_h / PH offset by the
    ROI start and clipped to the map; an empty bin gives 0 with Argmax -1."""
    x, rois = ctx.input("X"), ctx.input("ROIs")
    ph, pw, sc = ctx.attr("pooled_height"), ctx.attr("pooled_width"), ctx.attr("spatial_scale")
    if ctx.meta:
        shape = (rois.shape[0], x.shape[1], ph, pw)
        ctx.set_output("Out", torch.empty(shape, dtype=x.dtype, device="meta"))
        ctx.set_output("Argmax", torch.empty(shape, dtype=torch.int64, device="meta"))
        return
    batch_ids = _roi_batch_ids(ctx, rois)
    import math

    def rnd(v):
        return int(math.copysign(math.floor(abs(v) + 0.5), v))

    B, C, H, W = x.shape
    outs, args = [], []
    for i in range(rois.shape[0]):
        x1, y1, x2, y2 = [rnd(float(v) * sc) for v in rois[i].tolist()]
        rw, rh = max(x2 - x1 + 1, 1), max(y2 - y1 + 1, 1)
        o = torch.zeros(C, ph, pw, dtype=x.dtype, device=x.device)
        a = torch.full((C, ph, pw), -1, dtype=torch.int64, device=x.device)
        for py in range(ph):
            hs = min(max(math.floor(py * rh / ph) + y1, 0), H)
            he = min(max(math.ceil((py + 1) * rh / ph) + y1, 0), H)
            for px in range(pw):
                ws = min(max(math.floor(px * rw / pw) + x1, 0), W)
                we = min(max(math.ceil((px + 1) * rw / pw) + x1, 0), W)
                if he <= hs or we <= ws:
                    continue
                win = x[batch_ids[i], :, hs:he, ws:we].reshape(C, -1)
                m, j = win.max(1)
                o[:, py, px] = m
                a[:, py, px] = (j // (we - ws) + hs) * W + j % (we - ws) + ws
        outs.append(o)
        args.append(a)
    out = torch.stack(outs) if outs else torch.zeros(0, C, ph, pw, device=x.device, dtype=x.dtype)
    ctx.set_output("Out", out)
    ctx.set_output("Argmax", torch.stack(args) if args else torch.zeros(out.shape, dtype=torch.int64,
                                                                         device=x.device))


@register_op_kernel("roi_pool", "GPU", [torch.float32], library=LibraryType.NATIVE)
def roi_pool_native(ctx):
    """GPU kernel of roi_pool (seqdet.hip), fp32 as roi_pool_op.cu; other float
    types reach it through the data transform."""
    x, rois = ctx.input("X"), ctx.input("ROIs")
    r = _oplib.roi_pool_op(x, rois, _roi_batch_ids(ctx, rois), ctx.attr("pooled_height"), ctx.attr("pooled_width"),
                           ctx.attr("spatial_scale")) if rois.shape[0] else None
    if r is None:
        return roi_pool(ctx)
    ctx.set_output("Out", r[0])
    ctx.set_output("Argmax", r[1])


@register_op("row_conv", ["X", "Filter"], ["Out"], {})
def row_conv(ctx):
    """Lookahead conv over each sequence (row_conv_op.cu)."""
    x, w = ctx.input("X"), ctx.input("Filter")
    lod = ctx.input_lod("X")
    off = lod[0] if lod else [0, x.shape[0]]
    r = _oplib.row_conv_op(x, w, off) if x.is_cuda else None
    if r is not None:
        ctx.set_output("Out", r, lod)
        return
    out = torch.zeros_like(x)
    ctxlen = w.shape[0]
    for s, e in zip(off[:-1], off[1:]):
        seq = x[s:e]
        for k in range(ctxlen):
            if k >= e - s:
                break
            out[s:e - k] += seq[k:] * w[k]
    ctx.set_output("Out", out, lod)


@register_op("conv_shift", ["X", "Y"], ["Out"], {})
def conv_shift(ctx):
    x, y = ctx.input("X"), ctx.input("Y")
    from ..ops import nnmisc as _nm
    r = _nm.conv_shift(x, y)
    if r is not None:  # conv_shift kernels (nnmisc.hip)
        ctx.set_output("Out", r)
        return
    M, N = x.shape[1], y.shape[1]
    half = (N - 1) // 2
    idx = (torch.arange(M, device=x.device)[:, None] + torch.arange(N, device=x.device)[None, :] - half) % M
    ctx.set_output("Out", (x[:, idx] * y[:, None, :]).sum(-1))
