"""Runtime data model of the static-graph engine (the reference's L1 layer).

Parity: Place (platform/place.h:25-78), Tensor/LoDTensor
(framework/tensor.h:36, lod_tensor.h:58-149), SelectedRows (selected_rows.h:32),
Variable/Scope (variable.h:26, scope.h:39), LoDTensorArray, dtype enum
(framework.proto VarType.Type).

MI355X design: a tensor's storage is a PyTorch-ROCm tensor on ``cpu`` or
``cuda:N`` (the HIP device), so every kernel -- hand-written gfx950 HIP or
library -- works on it in place with no copies; LoD offsets stay host-side
Python lists (they drive shape logic, never device work).
"""
from __future__ import annotations

import threading
from collections import OrderedDict

import numpy as np
import torch

from .proto import VarTypeEnum as VT

# ------------------------------------------------------------------ dtypes

_NP2VT = {
    np.dtype("bool"): VT.BOOL, np.dtype("int16"): VT.INT16, np.dtype("int32"): VT.INT32,
    np.dtype("int64"): VT.INT64, np.dtype("float16"): VT.FP16, np.dtype("float32"): VT.FP32,
    np.dtype("float64"): VT.FP64, np.dtype("uint8"): VT.UINT8, np.dtype("int8"): VT.INT8,
}
_VT2TORCH = {
    VT.BOOL: torch.bool, VT.INT16: torch.int16, VT.INT32: torch.int32, VT.INT64: torch.int64,
    VT.FP16: torch.float16, VT.FP32: torch.float32, VT.FP64: torch.float64, VT.UINT8: torch.uint8,
    VT.INT8: torch.int8, VT.BF16: torch.bfloat16, VT.SIZE_T: torch.int64,
}
_TORCH2VT = {v: k for k, v in _VT2TORCH.items() if k != VT.SIZE_T}
_STR2VT = {"bool": VT.BOOL, "int16": VT.INT16, "int32": VT.INT32, "int64": VT.INT64, "float16": VT.FP16,
           "float32": VT.FP32, "float64": VT.FP64, "uint8": VT.UINT8, "int8": VT.INT8, "bfloat16": VT.BF16,
           "fp16": VT.FP16, "fp32": VT.FP32, "fp64": VT.FP64, "bf16": VT.BF16}
_VT_SIZE = {VT.BOOL: 1, VT.INT16: 2, VT.INT32: 4, VT.INT64: 8, VT.FP16: 2, VT.FP32: 4, VT.FP64: 8,
            VT.UINT8: 1, VT.INT8: 1, VT.BF16: 2, VT.SIZE_T: 8}


def convert_dtype(dtype) -> int:
    """Any of: VarType int, numpy dtype/str, torch dtype -> VarType int."""
    if dtype is None:
        return VT.FP32
    if isinstance(dtype, int):
        return dtype
    if isinstance(dtype, torch.dtype):
        return _TORCH2VT[dtype]
    if isinstance(dtype, str) and dtype in _STR2VT:
        return _STR2VT[dtype]
    return _NP2VT[np.dtype(dtype)]


def to_torch_dtype(vt) -> torch.dtype:
    return _VT2TORCH[convert_dtype(vt)]


def dtype_size(vt) -> int:
    return _VT_SIZE[convert_dtype(vt)]


def dtype_to_str(vt) -> str:
    vt = convert_dtype(vt)
    for k, v in _STR2VT.items():
        if v == vt and len(k) > 4:
            return k
    return {VT.FP16: "float16", VT.FP32: "float32", VT.FP64: "float64", VT.BF16: "bfloat16"}.get(vt, str(vt))


# ------------------------------------------------------------------ places


class Place:
    device: str = "cpu"

    def torch_device(self):
        return torch.device(self.device)

    def __eq__(self, o):
        return isinstance(o, Place) and self.torch_device() == o.torch_device() and type(self) is type(o)

    def __hash__(self):
        return hash((type(self).__name__, str(self.torch_device())))


class CPUPlace(Place):
    def __repr__(self):
        return "CPUPlace"


class CUDAPlace(Place):
    """The HIP device (the public name is kept for API parity)."""

    def __init__(self, device_id=0):
        self.device_id = int(device_id)
        self.device = f"cuda:{self.device_id}"

    def torch_device(self):
        return torch.device("cuda", self.device_id)

    def __repr__(self):
        return f"CUDAPlace({self.device_id})"


HIPPlace = CUDAPlace


class CUDAPinnedPlace(Place):
    def __repr__(self):
        return "CUDAPinnedPlace"


def is_compiled_with_cuda():
    return torch.cuda.is_available()


is_compiled_with_hip = is_compiled_with_cuda


def get_cuda_device_count():
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


def place_of(t: torch.Tensor) -> Place:
    return CUDAPlace(t.device.index or 0) if t.is_cuda else CPUPlace()


# ------------------------------------------------------------------ LoD helpers


def lengths_to_offsets(lengths):
    off = [0]
    for l in lengths:
        off.append(off[-1] + int(l))
    return off


def offsets_to_lengths(off):
    return [off[i + 1] - off[i] for i in range(len(off) - 1)]


def check_lod(lod, numel_rows=None):
    for lvl in lod:
        if len(lvl) < 1 or lvl[0] != 0 or any(lvl[i] > lvl[i + 1] for i in range(len(lvl) - 1)):
            return False
    for a, b in zip(lod[:-1], lod[1:]):
        if a[-1] != len(b) - 1:
            return False
    if numel_rows is not None and lod and lod[-1][-1] != numel_rows:
        return False
    return True


# ------------------------------------------------------------------ tensors


class LoDTensor:
    """Dense tensor + level-of-detail offsets (lod_tensor.h:110)."""

    __slots__ = ("_t", "_lod", "_layout")

    def __init__(self, tensor=None, lod=None, layout="AnyLayout"):
        self._t = tensor
        self._lod = [list(map(int, l)) for l in (lod or [])]
        self._layout = layout  # DataLayout tag read by the data transform (tensor.h layout_)

    @property
    def layout(self):
        return self._layout

    def set_layout(self, layout):
        self._layout = layout

    # -- storage
    @property
    def tensor(self):
        return self._t

    def set_tensor(self, t):
        self._t = t

    def set(self, array, place=None):
        if isinstance(array, torch.Tensor):
            t = array
        else:
            t = torch.from_numpy(np.ascontiguousarray(np.asarray(array)))
        dev = place.torch_device() if place is not None else (self._t.device if self._t is not None else "cpu")
        self._t = t.to(dev)

    def shape(self):
        return list(self._t.shape) if self._t is not None else []

    def _dtype(self):
        return convert_dtype(self._t.dtype)

    def _place(self):
        return place_of(self._t)

    def numel(self):
        return self._t.numel() if self._t is not None else 0

    def is_initialized(self):
        return self._t is not None

    # -- LoD (offset form)
    def lod(self):
        return [list(l) for l in self._lod]

    def set_lod(self, lod):
        self._lod = [list(map(int, l)) for l in lod]

    def recursive_sequence_lengths(self):
        return [offsets_to_lengths(l) for l in self._lod]

    def set_recursive_sequence_lengths(self, lens):
        self._lod = [lengths_to_offsets(l) for l in lens]

    def has_valid_recursive_sequence_lengths(self):
        rows = self._t.shape[0] if self._t is not None and self._t.dim() else None
        return check_lod(self._lod, rows)

    def lod_level(self):
        return len(self._lod)

    def numpy(self):
        t = self._t.detach()
        if t.dtype == torch.bfloat16:
            t = t.float()
        return t.cpu().numpy()

    def __array__(self, dtype=None, copy=None):
        a = self.numpy()
        return a.astype(dtype) if dtype is not None else a

    def __repr__(self):
        return f"LoDTensor(shape={self.shape()}, lod={self._lod})"


Tensor = LoDTensor


class SelectedRows:
    """Sparse rows {rows, height, value} (selected_rows.h:32-153)."""

    def __init__(self, rows=None, height=0, value=None):
        self._rows = list(rows or [])
        self._height = int(height)
        self._value = LoDTensor(value)

    def rows(self):
        return self._rows

    def set_rows(self, rows):
        self._rows = [int(r) for r in rows]

    def height(self):
        return self._height

    def set_height(self, h):
        self._height = int(h)

    def get_tensor(self):
        return self._value

    def to_dense(self):
        v = self._value.tensor
        out = torch.zeros((self._height,) + tuple(v.shape[1:]), dtype=v.dtype, device=v.device)
        if self._rows:
            idx = torch.as_tensor(self._rows, device=v.device, dtype=torch.long)
            out.index_add_(0, idx, v)
        return out


class LoDTensorArray(list):
    """Vector of LoDTensors (LOD_TENSOR_ARRAY)."""


class LoDRankTable:
    def __init__(self, items=None):
        self.items = items or []  # list of (index, length) sorted by length desc
        self.coarse_lod = []


# ------------------------------------------------------------------ variable / scope


class Variable:
    """Type-erased holder (variable.h:26)."""

    __slots__ = ("name", "_value")

    def __init__(self, name=None):
        self.name = name
        self._value = None

    def is_initialized(self):
        return self._value is not None

    def get(self):
        return self._value

    def set(self, v):
        self._value = v

    def get_tensor(self) -> LoDTensor:
        if self._value is None:
            self._value = LoDTensor()
        if isinstance(self._value, SelectedRows):
            return self._value.get_tensor()
        return self._value

    get_lod_tensor = get_tensor

    def get_selected_rows(self) -> SelectedRows:
        if self._value is None:
            self._value = SelectedRows()
        return self._value

    def get_lod_tensor_array(self) -> LoDTensorArray:
        if self._value is None:
            self._value = LoDTensorArray()
        return self._value

    def get_lod_rank_table(self):
        if self._value is None:
            self._value = LoDRankTable()
        return self._value

    def set_int(self, v):
        self._value = int(v)

    def get_int(self):
        return int(self._value)

    def set_float(self, v):
        self._value = float(v)

    def get_float(self):
        return float(self._value)

    def is_type(self, cls):
        return isinstance(self._value, cls)


class Scope:
    """Hierarchical name -> Variable map with kid scopes (scope.h:39)."""

    def __init__(self, parent=None):
        self._vars: "OrderedDict[str, Variable]" = OrderedDict()
        self._parent = parent
        self._kids = []
        self._lock = threading.Lock()

    def var(self, name) -> Variable:
        v = self._vars.get(name)
        if v is None:
            with self._lock:
                v = self._vars.get(name)
                if v is None:
                    v = Variable(name)
                    self._vars[name] = v
        return v

    def find_var(self, name):
        s = self
        while s is not None:
            v = s._vars.get(name)
            if v is not None:
                return v
            s = s._parent
        return None

    def find_local_var(self, name):
        return self._vars.get(name)

    def has_var(self, name):
        return self.find_var(name) is not None

    def erase(self, names):
        for n in names:
            self._vars.pop(n, None)

    def rename(self, old, new):
        v = self._vars.pop(old)
        v.name = new
        self._vars[new] = v

    def new_scope(self):
        s = Scope(self)
        self._kids.append(s)
        return s

    def drop_kids(self):
        self._kids = []

    def kids(self):
        return list(self._kids)

    def parent(self):
        return self._parent

    def local_var_names(self):
        return list(self._vars.keys())

    def __contains__(self, name):
        return self.has_var(name)


_global_scope = Scope()


def global_scope():
    return _global_scope


def _switch_scope(scope):
    global _global_scope
    old = _global_scope
    _global_scope = scope
    return old


class EOFException(Exception):
    """Raised when a reader is exhausted (reference platform/enforce.h EOFException,
    exposed as fluid.core.EOFException)."""
