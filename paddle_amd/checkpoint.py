"""``paddle.save`` / ``paddle.load``: ``.pdparams`` / ``.pdopt`` checkpoints.

Format (Paddle 2.x ``paddle.save`` of a state dict): a pickle (protocol 4) of a
dict whose tensors are stored as ``numpy.ndarray`` (nested dicts such as the
optimizer's ``LR_Scheduler`` entry are kept as-is); bf16 tensors are stored as
float32 arrays tagged in ``"__bf16_keys__"`` so they round-trip exactly.

Loading never executes code from the file: a restricted unpickler resolves only
numpy's array-reconstruction helpers, dtypes, ``OrderedDict`` and plain builtins;
any other global in the stream raises ``pickle.UnpicklingError``.

The static-graph checkpoint formats (LoDTensor streams per variable /
``save_combine``) live in ``fluid.io`` (reference python/paddle/fluid/io.py).
"""
from __future__ import annotations

import collections
import io
import os
import pickle

import numpy as np
import torch

_ALLOWED = {
    ("collections", "OrderedDict"),
    ("numpy", "ndarray"),
    ("numpy", "dtype"),
    ("numpy.core.multiarray", "_reconstruct"),
    ("numpy._core.multiarray", "_reconstruct"),
    ("numpy.core.multiarray", "scalar"),
    ("numpy._core.multiarray", "scalar"),
    ("_codecs", "encode"),
    ("builtins", "set"),
    ("builtins", "frozenset"),
    ("builtins", "slice"),
    ("builtins", "complex"),
}


class _SafeUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _ALLOWED or (module.startswith("numpy") and name.endswith("DType")):
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"global {module}.{name} is not allowed in a checkpoint")


def _to_np(obj, bf16_keys, prefix=""):
    if torch.is_tensor(obj):
        t = obj.detach().cpu()
        if t.dtype == torch.bfloat16:
            bf16_keys.append(prefix)
            t = t.float()
        return t.numpy()
    if isinstance(obj, dict):
        return type(obj)((k, _to_np(v, bf16_keys, f"{prefix}/{k}")) for k, v in obj.items()) \
            if isinstance(obj, collections.OrderedDict) else {k: _to_np(v, bf16_keys, f"{prefix}/{k}")
                                                               for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_np(v, bf16_keys, f"{prefix}/{i}") for i, v in enumerate(obj))
    return obj


def _from_np(obj, bf16, return_numpy, prefix=""):
    if isinstance(obj, np.ndarray):
        if return_numpy:
            return obj
        t = torch.from_numpy(np.ascontiguousarray(obj))
        return t.to(torch.bfloat16) if prefix in bf16 else t
    if isinstance(obj, dict):
        items = [(k, _from_np(v, bf16, return_numpy, f"{prefix}/{k}")) for k, v in obj.items() if k != "__bf16_keys__"]
        return collections.OrderedDict(items) if isinstance(obj, collections.OrderedDict) else dict(items)
    if isinstance(obj, (list, tuple)):
        return type(obj)(_from_np(v, bf16, return_numpy, f"{prefix}/{i}") for i, v in enumerate(obj))
    return obj


def save(obj, path, protocol=4, **configs):
    if hasattr(obj, "state_dict") and not isinstance(obj, dict):
        obj = obj.state_dict()
    bf16: list = []
    data = _to_np(obj, bf16)
    if isinstance(data, dict) and bf16:
        data = dict(data)
        data["__bf16_keys__"] = bf16
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        pickle.dump(data, f, protocol=protocol)
    os.replace(tmp, path)


def load(path, return_numpy=False, **configs):
    with open(path, "rb") as f:
        raw = f.read()
    data = _SafeUnpickler(io.BytesIO(raw)).load()
    bf16 = set(data.get("__bf16_keys__", [])) if isinstance(data, dict) else set()
    return _from_np(data, bf16, return_numpy)
