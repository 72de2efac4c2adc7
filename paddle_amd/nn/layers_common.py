"""paddle.nn layers: convolution, pooling, normalisation, activation, loss, misc.

Parameter names / shapes / defaults follow Paddle 2.x so ``.pdparams`` state dicts
load 1:1 (e.g. ``BatchNorm2D`` keeps ``weight``, ``bias``, ``_mean``,
``_variance``; ``Conv2D.weight`` is ``[out, in/groups, kh, kw]``; momentum 0.9
means ``running = 0.9 * running + 0.1 * batch``).
"""
from __future__ import annotations

import math

import torch

from . import functional as F
from . import initializer as I
from .layer import Layer, _to_torch_dtype


def _ntuple(v, n):
    return tuple(v) if isinstance(v, (list, tuple)) else (v,) * n


# ------------------------------------------------------------------ convolution
class _ConvNd(Layer):
    def __init__(self, nd, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 padding_mode="zeros", weight_attr=None, bias_attr=None, data_format="NCHW", transpose=False,
                 output_padding=0, dtype="float32"):
        super().__init__(None, dtype)
        self.nd, self.transpose = nd, transpose
        self._in, self._out = in_channels, out_channels
        self._kernel = _ntuple(kernel_size, nd)
        self._stride, self._padding, self._dilation = stride, padding, dilation
        self._groups, self._data_format, self._output_padding = groups, data_format, output_padding
        self._padding_mode = padding_mode
        if transpose:
            shape = [in_channels, out_channels // groups, *self._kernel]
        else:
            shape = [out_channels, in_channels // groups, *self._kernel]
        fan_in = (in_channels // groups) * math.prod(self._kernel)
        std = math.sqrt(2.0 / fan_in)
        self.weight = self.create_parameter(shape, weight_attr, default_initializer=I.Normal(0.0, std))
        self.bias = None if bias_attr is False else self.create_parameter([out_channels], bias_attr, is_bias=True)

    def extra_repr(self):
        return f"{self._in}, {self._out}, kernel_size={self._kernel}, stride={self._stride}, padding={self._padding}"


class Conv1D(_ConvNd):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 padding_mode="zeros", weight_attr=None, bias_attr=None, data_format="NCL"):
        super().__init__(1, in_channels, out_channels, kernel_size, stride, padding, dilation, groups, padding_mode,
                         weight_attr, bias_attr, data_format)

    def forward(self, x):
        return F.conv1d(x, self.weight, self.bias, self._stride, self._padding, self._dilation, self._groups,
                        self._data_format)


class Conv2D(_ConvNd):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 padding_mode="zeros", weight_attr=None, bias_attr=None, data_format="NCHW"):
        super().__init__(2, in_channels, out_channels, kernel_size, stride, padding, dilation, groups, padding_mode,
                         weight_attr, bias_attr, data_format)

    def forward(self, x):
        if self._padding_mode != "zeros":
            p = _ntuple(self._padding, 2)
            x = torch.nn.functional.pad(x, [p[1], p[1], p[0], p[0]], mode=self._padding_mode)
            return F.conv2d(x, self.weight, self.bias, self._stride, 0, self._dilation, self._groups,
                            self._data_format)
        return F.conv2d(x, self.weight, self.bias, self._stride, self._padding, self._dilation, self._groups,
                        self._data_format)


class Conv3D(_ConvNd):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 padding_mode="zeros", weight_attr=None, bias_attr=None, data_format="NCDHW"):
        super().__init__(3, in_channels, out_channels, kernel_size, stride, padding, dilation, groups, padding_mode,
                         weight_attr, bias_attr, data_format)

    def forward(self, x):
        return F.conv3d(x, self.weight, self.bias, self._stride, self._padding, self._dilation, self._groups)


class Conv2DTranspose(_ConvNd):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, output_padding=0, groups=1,
                 dilation=1, weight_attr=None, bias_attr=None, data_format="NCHW"):
        super().__init__(2, in_channels, out_channels, kernel_size, stride, padding, dilation, groups, "zeros",
                         weight_attr, bias_attr, data_format, transpose=True, output_padding=output_padding)

    def forward(self, x, output_size=None):
        return F.conv2d_transpose(x, self.weight, self.bias, self._stride, self._padding, self._output_padding,
                                  self._groups, self._dilation)


class Conv1DTranspose(_ConvNd):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, output_padding=0, groups=1,
                 dilation=1, weight_attr=None, bias_attr=None, data_format="NCL"):
        super().__init__(1, in_channels, out_channels, kernel_size, stride, padding, dilation, groups, "zeros",
                         weight_attr, bias_attr, data_format, transpose=True, output_padding=output_padding)

    def forward(self, x, output_size=None):
        return F.conv1d_transpose(x, self.weight, self.bias, self._stride, self._padding, self._output_padding,
                                  self._groups, self._dilation)


class Conv3DTranspose(_ConvNd):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, output_padding=0, groups=1,
                 dilation=1, weight_attr=None, bias_attr=None, data_format="NCDHW"):
        super().__init__(3, in_channels, out_channels, kernel_size, stride, padding, dilation, groups, "zeros",
                         weight_attr, bias_attr, data_format, transpose=True, output_padding=output_padding)

    def forward(self, x, output_size=None):
        return F.conv3d_transpose(x, self.weight, self.bias, self._stride, self._padding, self._output_padding,
                                  self._groups, self._dilation)


# ---------------------------------------------------------------------- pooling
class MaxPool2D(Layer):
    def __init__(self, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False,
                 data_format="NCHW", name=None):
        super().__init__(name)
        self.k, self.s, self.p, self.rm, self.cm, self.df = kernel_size, stride, padding, return_mask, ceil_mode, data_format

    def forward(self, x):
        return F.max_pool2d(x, self.k, self.s, self.p, self.rm, self.cm, self.df)


class AvgPool2D(Layer):
    def __init__(self, kernel_size, stride=None, padding=0, ceil_mode=False, exclusive=True, divisor_override=None,
                 data_format="NCHW", name=None):
        super().__init__(name)
        self.args = (kernel_size, stride, padding, ceil_mode, exclusive, divisor_override, data_format)

    def forward(self, x):
        return F.avg_pool2d(x, *self.args)


class MaxPool1D(Layer):
    def __init__(self, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False, name=None):
        super().__init__(name)
        self.args = (kernel_size, stride, padding, return_mask, ceil_mode)

    def forward(self, x):
        return F.max_pool1d(x, *self.args)


class AvgPool1D(Layer):
    def __init__(self, kernel_size, stride=None, padding=0, exclusive=True, ceil_mode=False, name=None):
        super().__init__(name)
        self.args = (kernel_size, stride, padding, exclusive, ceil_mode)

    def forward(self, x):
        return F.avg_pool1d(x, *self.args)


class MaxPool3D(Layer):
    def __init__(self, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False,
                 data_format="NCDHW", name=None):
        super().__init__(name)
        self.args = (kernel_size, stride, padding, return_mask, ceil_mode)

    def forward(self, x):
        return F.max_pool3d(x, *self.args)


class AvgPool3D(Layer):
    def __init__(self, kernel_size, stride=None, padding=0, ceil_mode=False, exclusive=True, divisor_override=None,
                 data_format="NCDHW", name=None):
        super().__init__(name)
        self.args = (kernel_size, stride, padding, ceil_mode, exclusive, divisor_override)

    def forward(self, x):
        return F.avg_pool3d(x, *self.args)


class AdaptiveAvgPool2D(Layer):
    def __init__(self, output_size, data_format="NCHW", name=None):
        super().__init__(name)
        self.os, self.df = output_size, data_format

    def forward(self, x):
        return F.adaptive_avg_pool2d(x, self.os, self.df)


class AdaptiveMaxPool2D(Layer):
    def __init__(self, output_size, return_mask=False, name=None):
        super().__init__(name)
        self.os, self.rm = output_size, return_mask

    def forward(self, x):
        return F.adaptive_max_pool2d(x, self.os, self.rm)


class AdaptiveAvgPool1D(Layer):
    def __init__(self, output_size, name=None):
        super().__init__(name)
        self.os = output_size

    def forward(self, x):
        return F.adaptive_avg_pool1d(x, self.os)


class AdaptiveAvgPool3D(Layer):
    def __init__(self, output_size, data_format="NCDHW", name=None):
        super().__init__(name)
        self.os = output_size

    def forward(self, x):
        return F.adaptive_avg_pool3d(x, self.os)


# ---------------------------------------------------------------- normalisation
class _BatchNormBase(Layer):
    def __init__(self, num_features, momentum=0.9, epsilon=1e-5, weight_attr=None, bias_attr=None,
                 data_format="NCHW", use_global_stats=None, name=None, dtype="float32"):
        super().__init__(name, dtype)
        self.weight = self.create_parameter([num_features], weight_attr, default_initializer=I.Constant(1.0))
        self.bias = self.create_parameter([num_features], bias_attr, is_bias=True)
        if weight_attr is False:
            self.weight.requires_grad_(False)
        if bias_attr is False:
            self.bias.requires_grad_(False)
        self.register_buffer("_mean", torch.zeros(num_features))
        self.register_buffer("_variance", torch.ones(num_features))
        self._momentum, self._epsilon = momentum, epsilon
        self._data_format, self._use_global_stats = data_format, use_global_stats
        for p in (self.weight, self.bias):
            p.no_weight_decay = True

    def forward(self, x):
        return F.batch_norm(x, self._mean, self._variance, self.weight, self.bias, self.training, self._momentum,
                            self._epsilon, self._data_format, self._use_global_stats)


class BatchNorm1D(_BatchNormBase):
    def __init__(self, num_features, momentum=0.9, epsilon=1e-5, weight_attr=None, bias_attr=None,
                 data_format="NCL", use_global_stats=None, name=None):
        super().__init__(num_features, momentum, epsilon, weight_attr, bias_attr,
                         "NCHW" if data_format in ("NC", "NCL") else "NHWC", use_global_stats, name)


class BatchNorm2D(_BatchNormBase):
    pass


class BatchNorm3D(_BatchNormBase):
    def __init__(self, num_features, momentum=0.9, epsilon=1e-5, weight_attr=None, bias_attr=None,
                 data_format="NCDHW", use_global_stats=None, name=None):
        super().__init__(num_features, momentum, epsilon, weight_attr, bias_attr,
                         "NCHW" if data_format == "NCDHW" else "NHWC", use_global_stats, name)


class BatchNorm(_BatchNormBase):
    """fluid.dygraph.BatchNorm signature (num_channels, act=...)."""

    def __init__(self, num_channels, act=None, is_test=False, momentum=0.9, epsilon=1e-5, param_attr=None,
                 bias_attr=None, dtype="float32", data_layout="NCHW", use_global_stats=False, **kw):
        super().__init__(num_channels, momentum, epsilon, param_attr, bias_attr, data_layout, use_global_stats,
                         dtype=dtype)
        self._act = act

    def forward(self, x):
        y = super().forward(x)
        return getattr(F, self._act)(y) if self._act else y


SyncBatchNorm = BatchNorm2D


class GroupNorm(Layer):
    def __init__(self, num_groups, num_channels, epsilon=1e-5, weight_attr=None, bias_attr=None,
                 data_format="NCHW", name=None):
        super().__init__(name)
        self.weight = self.create_parameter([num_channels], weight_attr, default_initializer=I.Constant(1.0))
        self.bias = self.create_parameter([num_channels], bias_attr, is_bias=True)
        self.g, self.eps = num_groups, epsilon

    def forward(self, x):
        return F.group_norm(x, self.g, self.eps, self.weight, self.bias)


class InstanceNorm2D(Layer):
    def __init__(self, num_features, epsilon=1e-5, momentum=0.9, weight_attr=None, bias_attr=None,
                 data_format="NCHW", name=None):
        super().__init__(name)
        self.scale = self.create_parameter([num_features], weight_attr, default_initializer=I.Constant(1.0))
        self.bias = self.create_parameter([num_features], bias_attr, is_bias=True)
        self.eps = epsilon

    def forward(self, x):
        return F.instance_norm(x, weight=self.scale, bias=self.bias, eps=self.eps)


InstanceNorm1D = InstanceNorm3D = InstanceNorm2D


class LocalResponseNorm(Layer):
    def __init__(self, size, alpha=1e-4, beta=0.75, k=1.0, data_format="NCHW", name=None):
        super().__init__(name)
        self.args = (size, alpha, beta, k)

    def forward(self, x):
        return F.local_response_norm(x, *self.args)


# ------------------------------------------------------------------ activations
def _act_layer(name, fn, **defaults):
    def __init__(self, *args, name=None, **kw):
        Layer.__init__(self, name)
        self._args = args
        self._kw = dict(defaults, **kw)

    def forward(self, x):
        return fn(x, *self._args, **self._kw)

    return type(name, (Layer,), {"__init__": __init__, "forward": forward})


ReLU = _act_layer("ReLU", F.relu)
ReLU6 = _act_layer("ReLU6", F.relu6)
LeakyReLU = _act_layer("LeakyReLU", F.leaky_relu)
ELU = _act_layer("ELU", F.elu)
SELU = _act_layer("SELU", F.selu)
CELU = _act_layer("CELU", F.celu)
GELU = _act_layer("GELU", F.gelu)
Silu = _act_layer("Silu", F.silu)
Swish = _act_layer("Swish", F.silu)
Mish = _act_layer("Mish", F.mish)
Sigmoid = _act_layer("Sigmoid", F.sigmoid)
Hardsigmoid = _act_layer("Hardsigmoid", F.hardsigmoid)
Hardswish = _act_layer("Hardswish", F.hardswish)
Hardtanh = _act_layer("Hardtanh", F.hardtanh)
Hardshrink = _act_layer("Hardshrink", F.hardshrink)
Softshrink = _act_layer("Softshrink", F.softshrink)
Tanhshrink = _act_layer("Tanhshrink", F.tanhshrink)
Softplus = _act_layer("Softplus", F.softplus)
Softsign = _act_layer("Softsign", F.softsign)
LogSigmoid = _act_layer("LogSigmoid", F.log_sigmoid)
Tanh = _act_layer("Tanh", F.tanh)
Softmax = _act_layer("Softmax", F.softmax)
LogSoftmax = _act_layer("LogSoftmax", F.log_softmax)
GLU = _act_layer("GLU", F.glu)


class PReLU(Layer):
    def __init__(self, num_parameters=1, init=0.25, weight_attr=None, data_format="NCHW", name=None):
        super().__init__(name)
        self.weight = self.create_parameter([num_parameters], weight_attr, default_initializer=I.Constant(init))
        self.df = data_format

    def forward(self, x):
        return F.prelu(x, self.weight, self.df)


class Maxout(Layer):
    def __init__(self, groups, axis=1, name=None):
        super().__init__(name)
        self.g, self.a = groups, axis

    def forward(self, x):
        return F.maxout(x, self.g, self.a)


# ------------------------------------------------------------------------ losses
class CrossEntropyLoss(Layer):
    def __init__(self, weight=None, ignore_index=-100, reduction="mean", soft_label=False, axis=-1,
                 use_softmax=True, label_smoothing=0.0, name=None):
        super().__init__(name)
        self.kw = dict(weight=weight, ignore_index=ignore_index, reduction=reduction, soft_label=soft_label,
                       axis=axis, use_softmax=use_softmax, label_smoothing=label_smoothing)

    def forward(self, input, label):
        return F.cross_entropy(input, label, **self.kw)


def _loss_layer(name, fn, argnames=("reduction",), defaults=("mean",)):
    def __init__(self, *args, name=None, **kw):
        Layer.__init__(self, name)
        self._kw = dict(zip(argnames, defaults))
        self._kw.update(dict(zip(argnames, args)))
        self._kw.update(kw)

    def forward(self, input, label, *extra):
        return fn(input, label, *extra, **self._kw)

    return type(name, (Layer,), {"__init__": __init__, "forward": forward})


MSELoss = _loss_layer("MSELoss", F.mse_loss)
L1Loss = _loss_layer("L1Loss", F.l1_loss)
NLLLoss = _loss_layer("NLLLoss", F.nll_loss, ("weight", "ignore_index", "reduction"), (None, -100, "mean"))
BCELoss = _loss_layer("BCELoss", F.binary_cross_entropy, ("weight", "reduction"), (None, "mean"))
BCEWithLogitsLoss = _loss_layer("BCEWithLogitsLoss", F.binary_cross_entropy_with_logits,
                                ("weight", "reduction", "pos_weight"), (None, "mean", None))
SmoothL1Loss = _loss_layer("SmoothL1Loss", F.smooth_l1_loss, ("reduction", "delta"), ("mean", 1.0))
KLDivLoss = _loss_layer("KLDivLoss", F.kl_div)
MarginRankingLoss = _loss_layer("MarginRankingLoss", F.margin_ranking_loss, ("margin", "reduction"), (0.0, "mean"))
HingeEmbeddingLoss = _loss_layer("HingeEmbeddingLoss", F.hinge_embedding_loss, ("margin", "reduction"),
                                 (1.0, "mean"))


class CTCLoss(Layer):
    def __init__(self, blank=0, reduction="mean"):
        super().__init__()
        self.blank, self.reduction = blank, reduction

    def forward(self, log_probs, labels, input_lengths, label_lengths, norm_by_times=False):
        return F.ctc_loss(log_probs, labels, input_lengths, label_lengths, self.blank, self.reduction)


# --------------------------------------------------------------------------- misc
class Identity(Layer):
    def forward(self, x):
        return x


class Flatten(Layer):
    def __init__(self, start_axis=1, stop_axis=-1):
        super().__init__()
        self.a, self.b = start_axis, stop_axis

    def forward(self, x):
        return torch.flatten(x, self.a, self.b)


class Upsample(Layer):
    def __init__(self, size=None, scale_factor=None, mode="nearest", align_corners=False, align_mode=0,
                 data_format="NCHW", name=None):
        super().__init__(name)
        self.args = (size, scale_factor, mode, align_corners)

    def forward(self, x):
        return F.interpolate(x, *self.args)


class Pad2D(Layer):
    def __init__(self, padding, mode="constant", value=0.0, data_format="NCHW", name=None):
        super().__init__(name)
        self.p = [padding] * 4 if isinstance(padding, int) else list(padding)
        self.mode, self.value = mode, value

    def forward(self, x):
        return F.pad(x, self.p, self.mode, self.value)


class PixelShuffle(Layer):
    def __init__(self, upscale_factor, data_format="NCHW", name=None):
        super().__init__(name)
        self.r = upscale_factor

    def forward(self, x):
        return F.pixel_shuffle(x, self.r)


class Bilinear(Layer):
    def __init__(self, in1_features, in2_features, out_features, weight_attr=None, bias_attr=None, name=None):
        super().__init__(name)
        self.weight = self.create_parameter([out_features, in1_features, in2_features], weight_attr)
        self.bias = None if bias_attr is False else self.create_parameter([1, out_features], bias_attr, is_bias=True)

    def forward(self, x1, x2):
        return F.bilinear(x1, x2, self.weight, self.bias)


class CosineSimilarity(Layer):
    def __init__(self, axis=1, eps=1e-8):
        super().__init__()
        self.a, self.eps = axis, eps

    def forward(self, x1, x2):
        return F.cosine_similarity(x1, x2, self.a, self.eps)


class ParameterList(Layer):
    def __init__(self, parameters=None):
        super().__init__()
        self._plist = torch.nn.ParameterList(parameters or [])

    def __getitem__(self, i):
        return self._plist[i]

    def __len__(self):
        return len(self._plist)

    def __iter__(self):
        return iter(self._plist)

    def append(self, p):
        self._plist.append(p)
        return self


class LayerDict(Layer):
    def __init__(self, sublayers=None):
        super().__init__()
        self._d = torch.nn.ModuleDict(sublayers or {})

    def __getitem__(self, k):
        return self._d[k]

    def __setitem__(self, k, v):
        self._d[k] = v

    def __len__(self):
        return len(self._d)

    def __iter__(self):
        return iter(self._d)

    def keys(self):
        return self._d.keys()

    def items(self):
        return self._d.items()

    def values(self):
        return self._d.values()


__all__ = [n for n in dir() if not n.startswith("_") and n[0].isupper()]
