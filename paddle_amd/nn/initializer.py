"""Parameter initializers (paddle.nn.initializer / fluid.initializer semantics).

Parity: python/paddle/fluid/initializer.py (Constant, Uniform, Normal,
TruncatedNormal, Xavier, MSRA, Bilinear).  These run eagerly on a tensor; the
static-graph path emits the equivalent fill/random ops into the startup program.
"""
from __future__ import annotations

import math

import torch


def _fans(t):
    if t.dim() < 2:
        return t.numel(), t.numel()
    if t.dim() == 2:  # paddle Linear [in, out]
        return t.shape[0], t.shape[1]
    rf = int(torch.tensor(t.shape[2:]).prod())
    return t.shape[1] * rf, t.shape[0] * rf  # conv [out, in, kh, kw]


class Initializer:
    def __call__(self, t):
        raise NotImplementedError


class Constant(Initializer):
    def __init__(self, value=0.0):
        self.value = value

    def __call__(self, t):
        with torch.no_grad():
            return t.fill_(self.value)


class Uniform(Initializer):
    def __init__(self, low=-1.0, high=1.0, seed=0):
        self.low, self.high = low, high

    def __call__(self, t):
        with torch.no_grad():
            return t.uniform_(self.low, self.high)


class Normal(Initializer):
    def __init__(self, mean=0.0, std=1.0, seed=0):
        self.mean, self.std = mean, std

    def __call__(self, t):
        with torch.no_grad():
            return t.normal_(self.mean, self.std)


class TruncatedNormal(Initializer):
    def __init__(self, mean=0.0, std=1.0, seed=0):
        self.mean, self.std = mean, std

    def __call__(self, t):
        with torch.no_grad():
            return torch.nn.init.trunc_normal_(t, self.mean, self.std, self.mean - 2 * self.std,
                                               self.mean + 2 * self.std)


class XavierUniform(Initializer):
    def __init__(self, fan_in=None, fan_out=None, gain=1.0):
        self.fi, self.fo, self.gain = fan_in, fan_out, gain

    def __call__(self, t):
        fi, fo = _fans(t)
        fi, fo = self.fi or fi, self.fo or fo
        lim = self.gain * math.sqrt(6.0 / (fi + fo))
        with torch.no_grad():
            return t.uniform_(-lim, lim)


class XavierNormal(XavierUniform):
    def __call__(self, t):
        fi, fo = _fans(t)
        fi, fo = self.fi or fi, self.fo or fo
        std = self.gain * math.sqrt(2.0 / (fi + fo))
        with torch.no_grad():
            return t.normal_(0, std)


class KaimingNormal(Initializer):
    def __init__(self, fan_in=None, negative_slope=0.0, nonlinearity="relu"):
        self.fi = fan_in

    def __call__(self, t):
        fi = self.fi or _fans(t)[0]
        with torch.no_grad():
            return t.normal_(0, math.sqrt(2.0 / fi))


class KaimingUniform(KaimingNormal):
    def __call__(self, t):
        fi = self.fi or _fans(t)[0]
        lim = math.sqrt(6.0 / fi)
        with torch.no_grad():
            return t.uniform_(-lim, lim)


class Bilinear(Initializer):
    """Bilinear upsampling kernel for conv_transpose weights [C, 1, K, K]."""

    def __call__(self, t):
        K = t.shape[-1]
        f = math.ceil(K / 2.0)
        c = (2 * f - 1 - f % 2) / (2.0 * f)
        og = torch.arange(K, dtype=torch.float32)
        w1 = 1 - (og / f - c).abs()
        w = torch.outer(w1, w1)
        with torch.no_grad():
            t.zero_()
            t[...] = w
        return t


# fluid aliases
ConstantInitializer = Constant
UniformInitializer = Uniform
NormalInitializer = Normal
TruncatedNormalInitializer = TruncatedNormal
XavierInitializer = XavierUniform
MSRAInitializer = KaimingNormal
BilinearInitializer = Bilinear
MSRA = KaimingNormal
Xavier = XavierUniform
