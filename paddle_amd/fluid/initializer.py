"""Static-graph initializers: each appends one fill/random op to the startup block.

Parity: python/paddle/fluid/initializer.py (Constant, Uniform, Normal, Xavier,
MSRA, Bilinear, NumpyArrayInitializer, force_init_on_cpu / init_on_cpu).
"""
from __future__ import annotations

import contextlib
import math

import numpy as np

from ..framework import core

_force_init_on_cpu_ = False


def force_init_on_cpu():
    return _force_init_on_cpu_


@contextlib.contextmanager
def init_on_cpu():
    global _force_init_on_cpu_
    pre = _force_init_on_cpu_
    _force_init_on_cpu_ = True
    try:
        yield
    finally:
        _force_init_on_cpu_ = pre


class Initializer:
    def __call__(self, param, block):
        raise NotImplementedError

    @staticmethod
    def _compute_fans(var):
        shape = var.shape
        if not shape or len(shape) == 0:
            return 1, 1
        if len(shape) == 1:
            return shape[0], shape[0]
        if len(shape) == 2:
            return shape[0], shape[1]
        rf = int(np.prod(shape[2:]))
        return shape[1] * rf, shape[0] * rf


class ConstantInitializer(Initializer):
    def __init__(self, value=0.0, force_cpu=False):
        self._value, self._force_cpu = value, force_cpu

    def __call__(self, var, block):
        return block.prepend_op(type="fill_constant", outputs={"Out": var},
                                attrs={"shape": list(var.shape), "dtype": var.dtype, "value": float(self._value),
                                       "force_cpu": self._force_cpu or force_init_on_cpu()})


class UniformInitializer(Initializer):
    def __init__(self, low=-1.0, high=1.0, seed=0):
        self._low, self._high, self._seed = low, high, seed

    def __call__(self, var, block):
        seed = self._seed or block.program.random_seed
        return block.prepend_op(type="uniform_random", outputs={"Out": var},
                                attrs={"shape": list(var.shape), "dtype": var.dtype, "min": self._low,
                                       "max": self._high, "seed": seed})


class NormalInitializer(Initializer):
    def __init__(self, loc=0.0, scale=1.0, seed=0):
        self._mean, self._std, self._seed = loc, scale, seed

    def __call__(self, var, block):
        seed = self._seed or block.program.random_seed
        return block.prepend_op(type="gaussian_random", outputs={"Out": var},
                                attrs={"shape": list(var.shape), "dtype": var.dtype, "mean": self._mean,
                                       "std": self._std, "seed": seed})


class TruncatedNormalInitializer(NormalInitializer):
    def __call__(self, var, block):
        seed = self._seed or block.program.random_seed
        return block.prepend_op(type="truncated_gaussian_random", outputs={"Out": var},
                                attrs={"shape": list(var.shape), "dtype": var.dtype, "mean": self._mean,
                                       "std": self._std, "seed": seed})


class XavierInitializer(Initializer):
    def __init__(self, uniform=True, fan_in=None, fan_out=None, seed=0):
        self._uniform, self._fan_in, self._fan_out, self._seed = uniform, fan_in, fan_out, seed

    def __call__(self, var, block):
        fi, fo = self._compute_fans(var)
        fi = self._fan_in if self._fan_in is not None else fi
        fo = self._fan_out if self._fan_out is not None else fo
        if self._uniform:
            lim = math.sqrt(6.0 / float(fi + fo))
            return UniformInitializer(-lim, lim, self._seed)(var, block)
        return NormalInitializer(0.0, math.sqrt(2.0 / float(fi + fo)), self._seed)(var, block)


class MSRAInitializer(Initializer):
    def __init__(self, uniform=True, fan_in=None, seed=0):
        self._uniform, self._fan_in, self._seed = uniform, fan_in, seed

    def __call__(self, var, block):
        fi, _ = self._compute_fans(var)
        fi = self._fan_in if self._fan_in is not None else fi
        if self._uniform:
            lim = math.sqrt(6.0 / float(fi))
            return UniformInitializer(-lim, lim, self._seed)(var, block)
        return NormalInitializer(0.0, math.sqrt(2.0 / float(fi)), self._seed)(var, block)


class BilinearInitializer(Initializer):
    def __call__(self, var, block):
        shape = var.shape
        if len(shape) != 4 or shape[2] != shape[3]:
            raise ValueError("Bilinear initializer needs a [C, 1, K, K] weight")
        K = shape[3]
        f = np.ceil(K / 2.0)
        c = (2 * f - 1 - f % 2) / (2.0 * f)
        w = np.zeros(shape, dtype=np.float32)
        for i in range(int(np.prod(shape))):
            x = i % K
            y = (i // K) % K
            w.flat[i] = (1 - abs(x / f - c)) * (1 - abs(y / f - c))
        return NumpyArrayInitializer(w)(var, block)


class NumpyArrayInitializer(Initializer):
    def __init__(self, value):
        self._value = np.asarray(value)

    def __call__(self, var, block):
        v = self._value
        if v.dtype in (np.float32, np.float64, np.float16):
            attrs = {"fp32_values": [float(x) for x in v.reshape(-1)]}
        else:
            attrs = {"int32_values": [int(x) for x in v.reshape(-1)]}
        attrs.update({"shape": list(v.shape), "dtype": var.dtype})
        return block.prepend_op(type="assign_value", outputs={"Out": var}, attrs=attrs)


Constant = ConstantInitializer
Uniform = UniformInitializer
Normal = NormalInitializer
TruncatedNormal = TruncatedNormalInitializer
Xavier = XavierInitializer
MSRA = MSRAInitializer
Bilinear = BilinearInitializer
