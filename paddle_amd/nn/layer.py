"""DyGraph ``Layer`` base and core layers (paddle.nn API surface).

Tensors are PyTorch-ROCm tensors; parameters use Paddle's layouts (``Linear``
weight is ``[in_features, out_features]``) so ``.pdparams`` state dicts map 1:1.
Hot math dispatches to the gfx950 kernels in :mod:`paddle_amd.ops`.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import torch

from ..utils import strict as _strict

from .. import ops
from ..autograd import engine as _eager
from . import initializer as I


class ParamBase(_eager.Tensor, torch.nn.Parameter):
    """DyGraph parameter: a framework ``Tensor`` (eager-engine leaf, stop_gradient
    False when trainable) that ``torch.nn.Module`` bookkeeping also registers as a
    parameter, with Paddle's writable ``name`` and ``trainable``."""

    @property
    def name(self):
        return self.__dict__.get("_pd_name")

    @name.setter
    def name(self, v):
        self.__dict__["_pd_name"] = v

    @property
    def trainable(self):
        return self.requires_grad

    @trainable.setter
    def trainable(self, v):
        self.requires_grad_(bool(v))

    def __deepcopy__(self, memo):
        p = ParamBase(self.data.clone(memory_format=torch.preserve_format), self.requires_grad)
        p.__dict__.update({k: v for k, v in self.__dict__.items()})
        memo[id(self)] = p
        return p

    def __reduce_ex__(self, proto):
        return (ParamBase, (self.data, self.requires_grad))


class Layer(torch.nn.Module):
    """Paddle-style layer: ``create_parameter``, ``parameters``, ``state_dict`` /
    ``set_state_dict``, ``train`` / ``eval``, ``full_name``."""

    _name_counter: dict = {}

    def __call__(self, *args, **kwargs):
        # one framework region per outermost layer call: every tensor op of the
        # forward runs inside it (native dispatch / strict accounting) without a
        # per-op region
        if not _strict.inside() and _strict.watching():
            with _strict.region("layer:" + type(self).__name__):
                return super().__call__(*args, **kwargs)
        return super().__call__(*args, **kwargs)

    def __init__(self, name_scope=None, dtype="float32"):
        super().__init__()
        base = name_scope or type(self).__name__.lower()
        n = Layer._name_counter.get(base, 0)
        Layer._name_counter[base] = n + 1
        self._full_name = f"{base}_{n}"
        self._dtype = dtype

    def full_name(self):
        return self._full_name

    def create_parameter(self, shape, attr=None, dtype=None, is_bias=False, default_initializer=None):
        dt = _to_torch_dtype(dtype or self._dtype)
        t = torch.empty(*shape, dtype=torch.float32)
        init = default_initializer
        if attr is not None and getattr(attr, "initializer", None) is not None:
            init = attr.initializer
        if init is None:
            init = I.Constant(0.0) if is_bias else I.XavierUniform()
        init(t)
        p = ParamBase(t.to(dt))
        if attr is not None and getattr(attr, "trainable", True) is False:
            p.requires_grad_(False)
        if attr is not None and getattr(attr, "name", None):
            p.name = attr.name
        else:  # Paddle's naming (<layer>.w_<k> / <layer>.b_<k>): keys of .pdopt accumulators
            kind = "b" if is_bias else "w"
            cnt = self.__dict__.setdefault("_pa_pcount", {})
            k = cnt.get(kind, 0)
            cnt[kind] = k + 1
            p.name = f"{self._full_name}.{kind}_{k}"
        return p

    def add_sublayer(self, name, sublayer):
        self.add_module(name, sublayer)
        return sublayer

    def sublayers(self, include_self=False):
        subs = [m for m in self.modules() if m is not self]
        return ([self] if include_self else []) + subs

    def named_sublayers(self, prefix="", include_self=False):
        for n, m in self.named_modules(prefix=prefix):
            if m is self and not include_self:
                continue
            yield n, m

    def add_parameter(self, name, parameter):
        self.register_parameter(name, parameter)
        return parameter

    def set_state_dict(self, state_dict, use_structured_name=True):
        own = self.state_dict().keys()
        missing = []
        with torch.no_grad():
            for k in own:
                if k in state_dict:
                    # the live tensor (state_dict() entries may be converted copies)
                    *path, attr = k.split(".")
                    mod = self.get_submodule(".".join(path)) if path else self
                    v = getattr(mod, attr)
                    src = state_dict[k]
                    if not torch.is_tensor(src):
                        src = torch.as_tensor(src)
                    conv = getattr(mod, "_pa_state_in", None)
                    if conv is not None:  # checkpoint layout -> in-memory layout
                        src = conv(attr, src)
                    v.copy_(src.to(v.dtype).view(v.shape))
                else:
                    missing.append(k)
        return missing, [k for k in state_dict if k not in own]

    set_dict = set_state_dict
    load_dict = set_state_dict

    def clear_gradients(self):
        for p in self.parameters():
            p.grad = None

    def to_static_state_dict(self):
        return OrderedDict((k, v.detach()) for k, v in self.state_dict().items())


def _to_torch_dtype(dt):
    if isinstance(dt, torch.dtype):
        return dt
    return {"float32": torch.float32, "float16": torch.float16, "bfloat16": torch.bfloat16,
            "float64": torch.float64, "fp32": torch.float32, "bf16": torch.bfloat16}[str(dt)]


class Linear(Layer):
    """y = x W + b, W: [in_features, out_features] (Paddle layout)."""

    def __init__(self, in_features, out_features, weight_attr=None, bias_attr=None, name=None,
                 dtype="float32", std=None):
        super().__init__(name, dtype)
        init = I.Normal(0.0, std) if std is not None else None
        self.weight = self.create_parameter([in_features, out_features], weight_attr,
                                            default_initializer=init)
        if bias_attr is False:
            self.bias = None
        else:
            self.bias = self.create_parameter([out_features], bias_attr, is_bias=True)
        self.in_features, self.out_features = in_features, out_features

    def forward(self, x):
        y = torch.matmul(x, self.weight)
        if self.bias is not None:
            y = y + self.bias
        return y


class Embedding(Layer):
    def __init__(self, num_embeddings, embedding_dim, padding_idx=None, sparse=False, weight_attr=None,
                 name=None, dtype="float32", std=None):
        super().__init__(name, dtype)
        init = I.Normal(0.0, std) if std is not None else I.XavierUniform()
        self.weight = self.create_parameter([num_embeddings, embedding_dim], weight_attr, default_initializer=init)
        self.padding_idx = padding_idx

    def forward(self, ids):
        return ops.embedding(ids, self.weight, self.padding_idx)


class RMSNorm(Layer):
    def __init__(self, hidden_size, epsilon=1e-6, dtype="float32", name=None):
        super().__init__(name, dtype)
        self.weight = self.create_parameter([hidden_size], default_initializer=I.Constant(1.0))
        self.epsilon = epsilon

    def forward(self, x, residual=None):
        return ops.rms_norm(x, self.weight, self.epsilon, residual=residual)


class LayerNorm(Layer):
    def __init__(self, normalized_shape, epsilon=1e-5, weight_attr=None, bias_attr=None, name=None,
                 dtype="float32"):
        super().__init__(name, dtype)
        n = normalized_shape if isinstance(normalized_shape, int) else int(math.prod(normalized_shape))
        self.weight = None if weight_attr is False else self.create_parameter([n], weight_attr,
                                                                              default_initializer=I.Constant(1.0))
        self.bias = None if bias_attr is False else self.create_parameter([n], bias_attr, is_bias=True)
        self.epsilon = epsilon
        self._n = n

    def forward(self, x, residual=None):
        return ops.layer_norm(x, self.weight, self.bias, self.epsilon, residual=residual)


class Dropout(Layer):
    def __init__(self, p=0.5, axis=None, mode="upscale_in_train", name=None):
        super().__init__(name)
        self.p, self.mode = p, mode

    def forward(self, x):
        if not self.training or self.p == 0:
            return x if self.mode == "upscale_in_train" else x * (1 - self.p)
        if self.mode == "upscale_in_train":
            return torch.nn.functional.dropout(x, self.p, True)
        return x * (torch.rand_like(x, dtype=torch.float32) >= self.p).to(x.dtype)


class Sequential(Layer):
    def __init__(self, *layers):
        super().__init__()
        for i, l in enumerate(layers):
            self.add_module(str(i), l)

    def forward(self, x):
        for l in self.children():
            x = l(x)
        return x


class LayerList(Layer):
    def __init__(self, sublayers=None):
        super().__init__()
        self._list = torch.nn.ModuleList(sublayers or [])

    def __getitem__(self, i):
        return self._list[i]

    def __len__(self):
        return len(self._list)

    def __iter__(self):
        return iter(self._list)

    def append(self, l):
        self._list.append(l)
        return self
