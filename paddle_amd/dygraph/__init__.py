"""fluid.dygraph (1.x imperative API) on the MI355X eager engine.

The reference snapshot has no imperative mode; this is the north-star
DyGraph layer: ``guard()`` selects the device, ``to_variable`` makes a tensor,
layers are :mod:`paddle_amd.nn` layers (1.x names ``Linear``/``FC``, ``Conv2D``,
``Pool2D``, ``BatchNorm``, ``Embedding``).  What runs where: tensor storage is a
PyTorch-ROCm tensor; autograd is the framework's own eager engine
(``autograd/engine.py``: recorded grad nodes with hand-written backward rules, no
torch.autograd); the hot ops (GEMM / linear, attention, norms, softmax-CE,
SwiGLU/GELU, embedding, AdamW/momentum, RoPE, NHWC conv / BN / pool) are fused
gfx950 kernels (``paddle_amd/csrc/kernels``), and the remaining pointwise / cast /
fill / reduction tensor ops issued inside the engine run on the generic HIP
kernels of ``csrc/kernels/tensor_ops.hip`` (``ops/aten_native.py``).  Whatever is
still an ATen kernel is counted per op by ``utils/strict.py`` and refused under
``FLAGS_strict_native=1``.
"""
from __future__ import annotations

import contextlib

import numpy as np
import torch

from .. import checkpoint as _ckpt
from .. import nn as _nn
from .. import tensor_api as _T
from ..distributed.parallel import DataParallel  # noqa: F401
from ..nn import BatchNorm, Embedding, Layer, LayerList, Sequential  # noqa: F401

_enabled = [False]


@contextlib.contextmanager
def guard(place=None):
    prev = _T._device[0]
    _enabled[0] = True
    if place is not None:
        _T._device[0] = _T._dev(place)
    try:
        yield
    finally:
        _enabled[0] = False
        _T._device[0] = prev


def enabled():
    return _enabled[0]


in_dygraph_mode = enabled


def enable_dygraph(place=None):
    _enabled[0] = True
    if place is not None:
        _T._device[0] = _T._dev(place)


def disable_dygraph():
    _enabled[0] = False


def to_variable(value, name=None, zero_copy=None, dtype=None):
    if torch.is_tensor(value):
        return value
    return _T.to_tensor(np.asarray(value), dtype=dtype)


no_grad = torch.no_grad


class Linear(_nn.Linear):
    """1.x ``Linear(input_dim, output_dim, param_attr, bias_attr, act, dtype)``."""

    def __init__(self, input_dim, output_dim, param_attr=None, bias_attr=None, act=None, dtype="float32"):
        super().__init__(input_dim, output_dim, param_attr, bias_attr, dtype=dtype)
        self._act = act

    def forward(self, x):
        y = super().forward(x)
        return getattr(_nn.functional, self._act)(y) if self._act else y


class FC(Linear):
    def __init__(self, name_scope=None, size=None, num_flatten_dims=1, param_attr=None, bias_attr=None, act=None,
                 is_test=False, dtype="float32", input_dim=None):
        self._lazy = input_dim is None
        self._size, self._nfd = size, num_flatten_dims
        self._cfg = (param_attr, bias_attr, act, dtype)
        if not self._lazy:
            super().__init__(input_dim, size, param_attr, bias_attr, act, dtype)
        else:
            Layer.__init__(self, name_scope)

    def forward(self, x):
        x2 = x.reshape(*x.shape[:self._nfd], -1) if x.dim() > self._nfd + 1 else x
        if self._lazy:
            pa, ba, act, dt = self._cfg
            Linear.__init__(self, x2.shape[-1], self._size, pa, ba, act, dt)
            self.to(x.device)
            self._lazy = False
        return super().forward(x2)


class Conv2D(_nn.Conv2D):
    """1.x ``Conv2D(num_channels, num_filters, filter_size, stride, padding, dilation, groups, ..., act)``."""

    def __init__(self, num_channels, num_filters, filter_size, stride=1, padding=0, dilation=1, groups=None,
                 param_attr=None, bias_attr=None, use_cudnn=True, act=None, dtype="float32"):
        super().__init__(num_channels, num_filters, filter_size, stride, padding, dilation, groups or 1,
                         weight_attr=param_attr, bias_attr=bias_attr)
        self._act = act

    def forward(self, x):
        y = super().forward(x)
        return getattr(_nn.functional, self._act)(y) if self._act else y


class Pool2D(Layer):
    def __init__(self, pool_size=-1, pool_type="max", pool_stride=1, pool_padding=0, global_pooling=False,
                 use_cudnn=True, ceil_mode=False, exclusive=True, data_format="NCHW"):
        super().__init__()
        self.args = (pool_size, pool_type, pool_stride, pool_padding, global_pooling, ceil_mode, exclusive)

    def forward(self, x):
        size, kind, stride, pad, glob, ceil, excl = self.args
        if glob:
            return _nn.functional.adaptive_avg_pool2d(x, 1) if kind == "avg" else \
                _nn.functional.adaptive_max_pool2d(x, 1)
        if kind == "max":
            return _nn.functional.max_pool2d(x, size, stride, pad, ceil_mode=ceil)
        return _nn.functional.avg_pool2d(x, size, stride, pad, ceil, excl)


def save_dygraph(state_dict, model_path):
    """``model_path`` + ``.pdparams`` (layer state) or ``.pdopt`` (optimizer state)."""
    is_opt = any(k in state_dict for k in ("LR_Scheduler", "global_step")) or any(
        "_moment" in k or "_velocity" in k or "_beta" in k for k in state_dict)
    _ckpt.save(state_dict, model_path + (".pdopt" if is_opt else ".pdparams"))


def load_dygraph(model_path, **configs):
    import os

    base = model_path[:-9] if model_path.endswith(".pdparams") else model_path
    params = _ckpt.load(base + ".pdparams") if os.path.exists(base + ".pdparams") else None
    opt = _ckpt.load(base + ".pdopt") if os.path.exists(base + ".pdopt") else None
    return params, opt


class BackwardStrategy:
    def __init__(self):
        self.sort_sum_gradient = False


def prepare_context(strategy=None):
    from ..parallel.comm import init_parallel_env

    init_parallel_env()
    return strategy


class ParallelEnv:
    @property
    def nranks(self):
        from ..parallel.comm import get_world_size

        return get_world_size()

    @property
    def local_rank(self):
        from ..parallel.comm import get_rank

        return get_rank()

    @property
    def dev_id(self):
        import os

        return int(os.environ.get("LOCAL_RANK", "0"))

    world_size = nranks
    rank = local_rank
