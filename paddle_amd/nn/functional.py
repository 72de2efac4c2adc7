"""``paddle.nn.functional`` on MI355X.

Hot paths dispatch to the hand-written gfx950 kernels in :mod:`paddle_amd.ops`
(softmax, softmax-cross-entropy, layer/RMS norm, rotary, SwiGLU, flash attention,
embedding); convolution / pooling / batch-norm go to MIOpen through PyTorch-ROCm
(NHWC bf16 when the input is channels-last).  Argument names and defaults follow
Paddle (``axis``, ``data_format="NCHW"``, ``epsilon``, ``[in, out]`` linear
weights, ``soft_label`` / ``ignore_index=-100`` cross entropy).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .. import ops
from ..ops import conv as _conv
from ..ops import convnd as _cnd


def _pair(v, n=2):
    return tuple(v) if isinstance(v, (list, tuple)) else (v,) * n


def _nchw(x, data_format):
    return data_format in ("NCHW", "NCL", "NCDHW")


# ------------------------------------------------------------------ activations
def relu(x, name=None):
    return F.relu(x)


def relu_(x, name=None):
    return F.relu_(x)


def relu6(x, name=None):
    return F.relu6(x)


def leaky_relu(x, negative_slope=0.01, name=None):
    return F.leaky_relu(x, negative_slope)


def elu(x, alpha=1.0, name=None):
    return F.elu(x, alpha)


def selu(x, scale=1.0507009873554804934193349852946, alpha=1.6732632423543772848170429916717, name=None):
    return scale * torch.where(x > 0, x, alpha * (torch.exp(x) - 1))


def celu(x, alpha=1.0, name=None):
    return F.celu(x, alpha)


def gelu(x, approximate=False, name=None):
    return F.gelu(x, approximate="tanh" if approximate else "none")


def silu(x, name=None):
    return F.silu(x)


swish = silu


def mish(x, name=None):
    return F.mish(x)


def sigmoid(x, name=None):
    return torch.sigmoid(x)


def hardsigmoid(x, slope=0.1666667, offset=0.5, name=None):
    return torch.clamp(x * slope + offset, 0.0, 1.0)


def hardswish(x, name=None):
    return F.hardswish(x)


def hardtanh(x, min=-1.0, max=1.0, name=None):
    return F.hardtanh(x, min, max)


def hardshrink(x, threshold=0.5, name=None):
    return F.hardshrink(x, threshold)


def softshrink(x, threshold=0.5, name=None):
    return F.softshrink(x, threshold)


def tanhshrink(x, name=None):
    return F.tanhshrink(x)


def softplus(x, beta=1, threshold=20, name=None):
    return F.softplus(x, beta, threshold)


def softsign(x, name=None):
    return F.softsign(x)


def log_sigmoid(x, name=None):
    return F.logsigmoid(x)


def tanh(x, name=None):
    return torch.tanh(x)


def prelu(x, weight, data_format="NCHW", name=None):
    if weight.numel() > 1 and not _nchw(x, data_format):
        return torch.where(x > 0, x, x * weight)
    return F.prelu(x, weight)


def maxout(x, groups, axis=1, name=None):
    s = list(x.shape)
    c = s[axis]
    s[axis:axis + 1] = [c // groups, groups]
    return x.reshape(s).max(dim=axis + 1)[0]


def glu(x, axis=-1, name=None):
    return F.glu(x, axis)


def swiglu(x, y=None, name=None):
    if y is not None:
        return F.silu(x) * y
    return ops.swiglu(x)


def softmax(x, axis=-1, dtype=None, name=None):
    if dtype is not None:
        x = x.to(_dt(dtype))
    if axis in (-1, x.dim() - 1) and x.dtype in (torch.float32, torch.bfloat16):
        return ops.softmax(x)
    return torch.softmax(x, axis)


def log_softmax(x, axis=-1, dtype=None, name=None):
    if dtype is not None:
        x = x.to(_dt(dtype))
    return torch.log_softmax(x, axis)


def _dt(d):
    from .layer import _to_torch_dtype

    return _to_torch_dtype(d)


# ----------------------------------------------------------------------- linear
def linear(x, weight, bias=None, name=None):
    """Paddle layout: ``weight`` is ``[in_features, out_features]``."""
    return ops.linear(x, weight, bias)


def bilinear(x1, x2, weight, bias=None, name=None):
    y = torch.einsum("bi,oij,bj->bo", x1, weight, x2)
    return y + bias if bias is not None else y


def embedding(x, weight, padding_idx=None, sparse=False, name=None):
    return ops.embedding(x, weight, padding_idx)


def one_hot(x, num_classes, name=None):
    return F.one_hot(x.long(), num_classes).float()


def dropout(x, p=0.5, axis=None, training=True, mode="upscale_in_train", name=None):
    if not training or p == 0:
        return x if mode == "upscale_in_train" else x * (1 - p)
    if axis is not None:
        axes = [axis] if isinstance(axis, int) else list(axis)
        shape = [x.shape[i] if i in axes else 1 for i in range(x.dim())]
        mask = (torch.rand(shape, device=x.device) >= p).to(x.dtype)
        return x * mask / (1 - p) if mode == "upscale_in_train" else x * mask
    if mode == "upscale_in_train":
        return F.dropout(x, p, True)
    return x * (torch.rand_like(x, dtype=torch.float32) >= p).to(x.dtype)


def dropout2d(x, p=0.5, training=True, data_format="NCHW", name=None):
    return dropout(x, p, axis=[0, 1] if _nchw(x, data_format) else [0, 3], training=training)


# ---------------------------------------------------------------- convolution
def _conv_padding(padding, nd):
    if isinstance(padding, str):
        return padding.lower()
    if isinstance(padding, int):
        return padding
    p = list(padding)
    if len(p) == nd:
        return tuple(p)
    if len(p) == 2 * nd:  # [before, after] per dim: symmetric only
        return tuple(p[0::2])
    return tuple(p)


def conv2d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NCHW", name=None):
    pad = _conv_padding(padding, 2)
    if (not _nchw(x, data_format) and groups > 1 and not isinstance(pad, str)
            and _conv.supported_dwconv(x, weight, groups)):
        return _conv.dwconv2d_nhwc(x, weight, bias, stride, pad, dilation)
    if not _nchw(x, data_format) and _conv.supported_conv(x, weight, stride, pad, dilation, groups):
        # NHWC bf16 on the GPU: implicit-GEMM MFMA kernel (ops/conv.py)
        return _conv.conv2d_nhwc(x, weight, bias, stride, pad, dilation)
    if not _nchw(x, data_format):
        y = F.conv2d(x.permute(0, 3, 1, 2), weight, bias, _pair(stride), pad, _pair(dilation), groups)
        return y.permute(0, 2, 3, 1)
    if not isinstance(pad, str) and _cnd.supported_conv(x, weight, groups):
        # NCHW on the GPU: vol2col + fp32 MFMA GEMM (ops/convnd.py)
        return _cnd.conv_nd(x, weight, bias, _pair(stride), pad, _pair(dilation), groups)
    return F.conv2d(x, weight, bias, _pair(stride), pad, _pair(dilation), groups)


def conv1d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NCL", name=None):
    pad = _conv_padding(padding, 1)
    if data_format == "NLC":
        return F.conv1d(x.transpose(1, 2), weight, bias, stride, pad, dilation, groups).transpose(1, 2)
    return F.conv1d(x, weight, bias, stride, pad, dilation, groups)


def conv3d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NCDHW", name=None):
    pad = _conv_padding(padding, 3)
    if data_format == "NCDHW" and not isinstance(pad, str) and _cnd.supported_conv(x, weight, groups):
        return _cnd.conv_nd(x, weight, bias, _pair(stride, 3), pad, _pair(dilation, 3), groups)
    return F.conv3d(x, weight, bias, _pair(stride, 3), _conv_padding(padding, 3), _pair(dilation, 3), groups)


def conv2d_transpose(x, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1, dilation=1,
                     data_format="NCHW", output_size=None, name=None):
    pad = _conv_padding(padding, 2)
    if _nchw(x, data_format) and not isinstance(pad, str) and _cnd.supported_conv_transpose(x, weight, groups):
        y = _cnd.conv_transpose_nd(x, weight, _pair(stride), pad, _pair(dilation), groups, _pair(output_padding))
        return y if bias is None else y + bias.to(y.dtype).reshape(1, -1, 1, 1)
    return F.conv_transpose2d(x, weight, bias, _pair(stride), _conv_padding(padding, 2), _pair(output_padding),
                              groups, _pair(dilation))


def conv1d_transpose(x, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1, dilation=1,
                     output_size=None, data_format="NCL", name=None):
    return F.conv_transpose1d(x, weight, bias, stride, padding, output_padding, groups, dilation)


def conv3d_transpose(x, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1, dilation=1,
                     data_format="NCDHW", output_size=None, name=None):
    return F.conv_transpose3d(x, weight, bias, _pair(stride, 3), _conv_padding(padding, 3),
                              _pair(output_padding, 3), groups, _pair(dilation, 3))


# ---------------------------------------------------------------------- pooling
def max_pool2d(x, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False, data_format="NCHW",
               name=None):
    stride = kernel_size if stride is None else stride
    if not _nchw(x, data_format) and not return_mask and _conv.supported_pool(x, ceil_mode) \
            and not isinstance(padding, str):
        return _conv.max_pool2d_nhwc(x, kernel_size, stride, _conv_padding(padding, 2))
    if _nchw(x, data_format) and not isinstance(padding, str) and _cnd.supported_pool(x) and x.dim() == 4:
        return _cnd.pool_nd(x, "max", _pair(kernel_size), _pair(stride), _conv_padding(padding, 2),
                            ceil_mode=ceil_mode, return_mask=return_mask)
    if not _nchw(x, data_format):
        x = x.permute(0, 3, 1, 2)
    y = F.max_pool2d(x, _pair(kernel_size), _pair(stride), _conv_padding(padding, 2), ceil_mode=ceil_mode,
                     return_indices=return_mask)
    if not _nchw(x, data_format):
        y = y.permute(0, 2, 3, 1) if not return_mask else (y[0].permute(0, 2, 3, 1), y[1].permute(0, 2, 3, 1))
    return y


def avg_pool2d(x, kernel_size, stride=None, padding=0, ceil_mode=False, exclusive=True, divisor_override=None,
               data_format="NCHW", name=None):
    stride = kernel_size if stride is None else stride
    nchw = _nchw(x, data_format)
    if nchw and divisor_override is None and not isinstance(padding, str) and _cnd.supported_pool(x) \
            and x.dim() == 4:
        return _cnd.pool_nd(x, "avg", _pair(kernel_size), _pair(stride), _conv_padding(padding, 2), exclusive,
                            ceil_mode)
    if not nchw:
        x = x.permute(0, 3, 1, 2)
    y = F.avg_pool2d(x, _pair(kernel_size), _pair(stride), _conv_padding(padding, 2), ceil_mode,
                     count_include_pad=not exclusive, divisor_override=divisor_override)
    return y if nchw else y.permute(0, 2, 3, 1)


def max_pool1d(x, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False, name=None):
    return F.max_pool1d(x, kernel_size, kernel_size if stride is None else stride, padding, ceil_mode=ceil_mode,
                        return_indices=return_mask)


def avg_pool1d(x, kernel_size, stride=None, padding=0, exclusive=True, ceil_mode=False, name=None):
    return F.avg_pool1d(x, kernel_size, kernel_size if stride is None else stride, padding, ceil_mode,
                        count_include_pad=not exclusive)


def max_pool3d(x, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False, data_format="NCDHW",
               name=None):
    if data_format == "NCDHW" and not isinstance(padding, str) and _cnd.supported_pool(x) and x.dim() == 5:
        return _cnd.pool_nd(x, "max", _pair(kernel_size, 3), _pair(kernel_size if stride is None else stride, 3),
                            _conv_padding(padding, 3), ceil_mode=ceil_mode, return_mask=return_mask)
    return F.max_pool3d(x, kernel_size, kernel_size if stride is None else stride, padding, ceil_mode=ceil_mode,
                        return_indices=return_mask)


def avg_pool3d(x, kernel_size, stride=None, padding=0, ceil_mode=False, exclusive=True, divisor_override=None,
               data_format="NCDHW", name=None):
    if (data_format == "NCDHW" and divisor_override is None and not isinstance(padding, str)
            and _cnd.supported_pool(x) and x.dim() == 5):
        return _cnd.pool_nd(x, "avg", _pair(kernel_size, 3), _pair(kernel_size if stride is None else stride, 3),
                            _conv_padding(padding, 3), exclusive, ceil_mode)
    return F.avg_pool3d(x, kernel_size, kernel_size if stride is None else stride, padding, ceil_mode,
                        count_include_pad=not exclusive, divisor_override=divisor_override)


def adaptive_avg_pool2d(x, output_size, data_format="NCHW", name=None):
    if not _nchw(x, data_format) and tuple(_pair(output_size)) == (1, 1) and _conv.supported_pool(x):
        return _conv.global_avg_pool_nhwc(x)
    if not _nchw(x, data_format):
        return F.adaptive_avg_pool2d(x.permute(0, 3, 1, 2), output_size).permute(0, 2, 3, 1)
    return F.adaptive_avg_pool2d(x, output_size)


def adaptive_max_pool2d(x, output_size, return_mask=False, name=None):
    return F.adaptive_max_pool2d(x, output_size, return_mask)


def adaptive_avg_pool1d(x, output_size, name=None):
    return F.adaptive_avg_pool1d(x, output_size)


def adaptive_max_pool1d(x, output_size, return_mask=False, name=None):
    return F.adaptive_max_pool1d(x, output_size, return_mask)


def adaptive_avg_pool3d(x, output_size, data_format="NCDHW", name=None):
    return F.adaptive_avg_pool3d(x, output_size)


# ---------------------------------------------------------------- normalisation
def batch_norm(x, running_mean, running_var, weight, bias, training=False, momentum=0.9, epsilon=1e-5,
               data_format="NCHW", use_global_stats=None, name=None):
    """Paddle momentum convention: running = running * momentum + batch * (1 - momentum)."""
    if use_global_stats:
        training = False
    if x.dim() == 4 and not _nchw(x, data_format) and _conv.supported_bn(x):
        if training:
            return _conv.batch_norm_nhwc_train(x, weight, bias, running_mean, running_var, momentum, epsilon)
        return _conv.batch_norm_nhwc_eval(x, weight, bias, running_mean, running_var, epsilon)
    nchw = _nchw(x, data_format) or x.dim() == 2
    if (nchw and x.dim() >= 2 and _cnd.supported_bn(x) and weight is not None and bias is not None
            and running_mean is not None and running_var is not None):
        # channel-first on the GPU: convnd.hip batch norm (no MIOpen)
        y, mo, vo, _, _ = _cnd.batch_norm_nchw(x, weight, bias, running_mean, running_var, momentum, epsilon,
                                               training, unbiased_running_var=True)
        if training:
            with torch.no_grad():
                running_mean.copy_(mo)
                running_var.copy_(vo)
        return y
    if not nchw:
        x = x.movedim(-1, 1)
    y = F.batch_norm(x, running_mean, running_var, weight, bias, training, 1.0 - momentum, epsilon)
    return y if nchw else y.movedim(1, -1)


def layer_norm(x, normalized_shape, weight=None, bias=None, epsilon=1e-5, name=None):
    n = normalized_shape if isinstance(normalized_shape, int) else int(math.prod(normalized_shape))
    if weight is not None and (x.is_cuda or True) and n == x.shape[-1]:
        return ops.layer_norm(x, weight, bias, epsilon)
    ns = [normalized_shape] if isinstance(normalized_shape, int) else list(normalized_shape)
    return F.layer_norm(x, ns, weight, bias, epsilon)


def rms_norm(x, weight, epsilon=1e-6, residual=None, name=None):
    return ops.rms_norm(x, weight, epsilon, residual=residual)


def instance_norm(x, running_mean=None, running_var=None, weight=None, bias=None, use_input_stats=True,
                  momentum=0.9, eps=1e-5, data_format="NCHW", name=None):
    return F.instance_norm(x, running_mean, running_var, weight, bias, use_input_stats, 1 - momentum, eps)


def group_norm(x, num_groups, epsilon=1e-5, weight=None, bias=None, data_format="NCHW", name=None):
    return F.group_norm(x, num_groups, weight, bias, epsilon)


def local_response_norm(x, size, alpha=1e-4, beta=0.75, k=1.0, data_format="NCHW", name=None):
    return F.local_response_norm(x, size, alpha, beta, k)


def normalize(x, p=2, axis=1, epsilon=1e-12, name=None):
    return F.normalize(x, p, axis, epsilon)


# ------------------------------------------------------------------------ losses
def _reduce(loss, reduction):
    if reduction == "mean":
        return loss.mean()
    if reduction == "sum":
        return loss.sum()
    return loss


def cross_entropy(input, label, weight=None, ignore_index=-100, reduction="mean", soft_label=False, axis=-1,
                  use_softmax=True, label_smoothing=0.0, name=None):
    if axis not in (-1, input.dim() - 1):
        input = input.movedim(axis, -1)
        label = label.movedim(axis, -1) if soft_label else label
    C = input.shape[-1]
    if soft_label:
        logp = torch.log_softmax(input.float(), -1) if use_softmax else torch.log(input.float())
        loss = -(label.float() * logp).sum(-1)
        return _reduce(loss, reduction)
    lab = label.reshape(input.shape[:-1]) if label.dim() == input.dim() else label
    lab = lab.long()
    if use_softmax and weight is None and label_smoothing == 0.0 and input.dtype in (torch.float32, torch.bfloat16):
        loss = ops.softmax_cross_entropy(input.reshape(-1, C), lab.reshape(-1), ignore_index=ignore_index,
                                         reduction="none").reshape(lab.shape)
        if reduction == "mean":
            return loss.sum() / (lab != ignore_index).sum().clamp(min=1)
        return _reduce(loss, reduction)
    x = input.reshape(-1, C).float()
    if not use_softmax:
        x = torch.log(x)
        return F.nll_loss(x, lab.reshape(-1), weight, ignore_index=ignore_index, reduction=reduction)
    return F.cross_entropy(x, lab.reshape(-1), weight, ignore_index=ignore_index, reduction=reduction,
                           label_smoothing=label_smoothing).reshape(lab.shape if reduction == "none" else ())


def softmax_with_cross_entropy(logits, label, soft_label=False, ignore_index=-100, numeric_stable_mode=True,
                               return_softmax=False, axis=-1):
    loss = cross_entropy(logits, label, soft_label=soft_label, ignore_index=ignore_index, reduction="none",
                         axis=axis).unsqueeze(-1)
    if return_softmax:
        return loss, torch.softmax(logits, axis)
    return loss


def nll_loss(input, label, weight=None, ignore_index=-100, reduction="mean", name=None):
    return F.nll_loss(input, label.long(), weight, ignore_index=ignore_index, reduction=reduction)


def mse_loss(input, label, reduction="mean", name=None):
    return F.mse_loss(input, label, reduction=reduction)


def l1_loss(input, label, reduction="mean", name=None):
    return F.l1_loss(input, label, reduction=reduction)


def smooth_l1_loss(input, label, reduction="mean", delta=1.0, name=None):
    return F.huber_loss(input, label, reduction=reduction, delta=delta)


def binary_cross_entropy(input, label, weight=None, reduction="mean", name=None):
    return F.binary_cross_entropy(input, label, weight, reduction=reduction)


def binary_cross_entropy_with_logits(logit, label, weight=None, reduction="mean", pos_weight=None, name=None):
    return F.binary_cross_entropy_with_logits(logit, label, weight, reduction=reduction, pos_weight=pos_weight)


def kl_div(input, label, reduction="mean", name=None):
    return F.kl_div(input, label, reduction="batchmean" if reduction == "batchmean" else reduction)


def margin_ranking_loss(input, other, label, margin=0.0, reduction="mean", name=None):
    return F.margin_ranking_loss(input, other, label, margin, reduction=reduction)


def hinge_embedding_loss(input, label, margin=1.0, reduction="mean", name=None):
    return F.hinge_embedding_loss(input, label, margin, reduction=reduction)


def cosine_similarity(x1, x2, axis=1, eps=1e-8):
    return F.cosine_similarity(x1, x2, axis, eps)


def ctc_loss(log_probs, labels, input_lengths, label_lengths, blank=0, reduction="mean", norm_by_times=False):
    return F.ctc_loss(log_probs, labels, input_lengths, label_lengths, blank, reduction=reduction)


def label_smooth(label, prior_dist=None, epsilon=0.1, name=None):
    C = label.shape[-1]
    p = prior_dist if prior_dist is not None else torch.full_like(label, 1.0 / C)
    return (1 - epsilon) * label + epsilon * p


# ------------------------------------------------------------------- attention
def scaled_dot_product_attention(query, key, value, attn_mask=None, dropout_p=0.0, is_causal=False,
                                 training=True, name=None):
    """[B, S, H, D] (Paddle layout)."""
    if attn_mask is None and dropout_p == 0.0:
        return ops.flash_attention(query, key, value, causal=is_causal)
    q, k, v = (t.transpose(1, 2) for t in (query, key, value))
    o = F.scaled_dot_product_attention(q, k, v, attn_mask, dropout_p if training else 0.0, is_causal)
    return o.transpose(1, 2)


def flash_attention(query, key, value, dropout=0.0, causal=False, return_softmax=False, training=True, name=None):
    return ops.flash_attention(query, key, value, causal=causal), None


def fused_rotary_position_embedding(q, k=None, v=None, sin=None, cos=None, position_ids=None,
                                    use_neox_rotary_style=True):
    out = [ops.apply_rotary(q, cos, sin)]
    if k is not None:
        out.append(ops.apply_rotary(k, cos, sin))
    if v is not None:
        out.append(v)
    return tuple(out)


# ------------------------------------------------------------------------ misc
def pad(x, pad, mode="constant", value=0.0, data_format="NCHW", name=None):
    return F.pad(x, list(pad), mode, value)


def interpolate(x, size=None, scale_factor=None, mode="nearest", align_corners=False, align_mode=0,
                data_format="NCHW", name=None):
    return F.interpolate(x, size, scale_factor, mode, align_corners if mode in ("linear", "bilinear", "bicubic",
                                                                                "trilinear") else None)


upsample = interpolate


def pixel_shuffle(x, upscale_factor, data_format="NCHW", name=None):
    return F.pixel_shuffle(x, upscale_factor)


def unfold(x, kernel_sizes, strides=1, paddings=0, dilations=1, name=None):
    return F.unfold(x, kernel_sizes, dilations, paddings, strides)


def fold(x, output_sizes, kernel_sizes, strides=1, paddings=0, dilations=1, name=None):
    return F.fold(x, output_sizes, kernel_sizes, dilations, paddings, strides)


def grid_sample(x, grid, mode="bilinear", padding_mode="zeros", align_corners=True, name=None):
    return F.grid_sample(x, grid, mode, padding_mode, align_corners)


def affine_grid(theta, out_shape, align_corners=True, name=None):
    return F.affine_grid(theta, list(out_shape), align_corners)
