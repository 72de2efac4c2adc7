"""``paddle.*`` tensor functions (creation, math, manipulation, logic, search,
random, linalg) with Paddle 2.x signatures.

Every tensor these functions return is the framework's ``paddle.Tensor``
(``autograd/engine.py``): storage and kernels are the PyTorch-ROCm tensor it
wraps, gradients come from the framework's own eager engine (explicit backward
rules, no torch autograd).  The functions map Paddle's signatures (``axis`` /
``keepdim`` / ``num_or_sections`` / ``perm`` ...) onto the kernels.
"""
from __future__ import annotations

import builtins
import math

import numpy as np
import torch

from .autograd import engine as _eager
from .nn.layer import _to_torch_dtype

Tensor = _eager.Tensor

_DT = {"float32": torch.float32, "float64": torch.float64, "float16": torch.float16, "bfloat16": torch.bfloat16,
       "int64": torch.int64, "int32": torch.int32, "int16": torch.int16, "int8": torch.int8, "uint8": torch.uint8,
       "bool": torch.bool, "complex64": torch.complex64, "complex128": torch.complex128,
       "float8_e4m3fn": torch.float8_e4m3fn, "float8_e5m2": torch.float8_e5m2}
_default_dtype = [torch.float32]
_device = [None]


def _dtype(d):
    if d is None:
        return None
    if isinstance(d, torch.dtype):
        return d
    if isinstance(d, np.dtype) or (isinstance(d, type) and issubclass(d, np.generic)):
        return torch.from_numpy(np.zeros(0, dtype=d)).dtype
    return _DT[str(d).replace("paddle.", "")]


def set_default_dtype(d):
    _default_dtype[0] = _dtype(d)


def get_default_dtype():
    return str(_default_dtype[0]).replace("torch.", "")


def _dev(place=None):
    if place is not None:
        if isinstance(place, str):
            return torch.device("cuda:0" if place in ("gpu", "hip") else place.replace("gpu", "cuda"))
        d = getattr(place, "torch_device", None)
        return d() if callable(d) else torch.device(d)
    if _device[0] is not None:
        return _device[0]
    return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


def set_device(device):
    """'cpu' | 'gpu' | 'gpu:N' (also 'hip:N')."""
    d = str(device).replace("hip", "cuda").replace("gpu", "cuda")
    _device[0] = torch.device(d)
    if _device[0].type == "cuda":
        torch.cuda.set_device(_device[0].index or 0)
    return _device[0]


def get_device():
    d = _dev()
    return "cpu" if d.type == "cpu" else f"gpu:{d.index or 0}"


def is_compiled_with_cuda():
    return torch.cuda.is_available()


is_compiled_with_rocm = is_compiled_with_cuda


# ----------------------------------------------------------------------- creation
def to_tensor(data, dtype=None, place=None, stop_gradient=True):
    dt = _dtype(dtype)
    if torch.is_tensor(data):
        t = data.detach().clone()
    else:
        arr = np.asarray(data)
        if dt is None and arr.dtype == np.float64 and not isinstance(data, np.ndarray):
            arr = arr.astype(np.float32)
        t = torch.from_numpy(np.ascontiguousarray(arr)) if arr.dtype != object else torch.tensor(data)
    if dt is None and t.dtype == torch.float64 and not isinstance(data, (np.ndarray, torch.Tensor)):
        dt = _default_dtype[0]
    with torch._C.DisableTorchFunctionSubclass():
        t = t.to(device=_dev(place), dtype=dt or t.dtype)
    return _eager.to_tensor_handle(t, stop_gradient=stop_gradient)


def _shape(s):
    if torch.is_tensor(s):
        return [int(x) for x in s.reshape(-1).tolist()]
    return [int(x) if not torch.is_tensor(x) else int(x.item()) for x in ([s] if isinstance(s, int) else s)]


def _filled(shape, value, dtype, device):
    """A new tensor of ``value``: on a GPU the framework's fill kernel (ops/oplib.py ->
    tensor_ops.hip / csrc/fastops), no ATen fill."""
    dev = torch.device(device) if device is not None else torch.device("cpu")
    if dev.type == "cuda" and not isinstance(value, complex):
        from .ops import oplib

        with torch._C.DisableTorchFunctionSubclass():
            return oplib.fill_(torch.empty(shape, dtype=dtype, device=dev), value)
    return torch.full(shape, value, dtype=dtype, device=dev)


def _filled_like(x, value, dtype):
    dt = _dtype(dtype) or x.dtype
    if x.is_cuda and not isinstance(value, complex):
        from .ops import oplib

        # empty_like keeps x's memory format (channels-last stays channels-last)
        with torch._C.DisableTorchFunctionSubclass():
            return oplib.fill_(torch.empty_like(x, dtype=dt), value)
    return torch.full_like(x, value, dtype=dt)


def zeros(shape, dtype=None, name=None):
    return _filled(_shape(shape), 0, _dtype(dtype) or _default_dtype[0], _dev())


def ones(shape, dtype=None, name=None):
    return _filled(_shape(shape), 1, _dtype(dtype) or _default_dtype[0], _dev())


def full(shape, fill_value, dtype=None, name=None):
    if torch.is_tensor(fill_value):
        fill_value = fill_value.item()
    return _filled(_shape(shape), fill_value, _dtype(dtype) or _default_dtype[0], _dev())


def empty(shape, dtype=None, name=None):
    return torch.empty(_shape(shape), dtype=_dtype(dtype) or _default_dtype[0], device=_dev())


def zeros_like(x, dtype=None, name=None):
    return _filled_like(x, 0, dtype)


def ones_like(x, dtype=None, name=None):
    return _filled_like(x, 1, dtype)


def full_like(x, fill_value, dtype=None, name=None):
    if torch.is_tensor(fill_value):
        fill_value = fill_value.item()
    return _filled_like(x, fill_value, dtype)


def empty_like(x, dtype=None, name=None):
    return torch.empty_like(x, dtype=_dtype(dtype))


def arange(start=0, end=None, step=1, dtype=None, name=None):
    if end is None:
        start, end = 0, start
    dt = _dtype(dtype) or (torch.int64 if builtins.all(isinstance(v, int) for v in (start, end, step)) else _default_dtype[0])
    return torch.arange(start, end, step, dtype=dt, device=_dev())


def linspace(start, stop, num, dtype=None, name=None):
    return torch.linspace(start, stop, num, dtype=_dtype(dtype) or _default_dtype[0], device=_dev())


def logspace(start, stop, num, base=10.0, dtype=None, name=None):
    return torch.logspace(start, stop, num, base, dtype=_dtype(dtype) or _default_dtype[0], device=_dev())


def eye(num_rows, num_columns=None, dtype=None, name=None):
    return torch.eye(num_rows, num_columns or num_rows, dtype=_dtype(dtype) or _default_dtype[0], device=_dev())


def diag(x, offset=0, padding_value=0, name=None):
    return torch.diag(x, offset)


def diagflat(x, offset=0, name=None):
    return torch.diagflat(x, offset)


def meshgrid(*args, **kw):
    if len(args) == 1 and isinstance(args[0], (list, tuple)):
        args = args[0]
    return list(torch.meshgrid(*args, indexing="ij"))


def tril(x, diagonal=0, name=None):
    return torch.tril(x, diagonal)


def triu(x, diagonal=0, name=None):
    return torch.triu(x, diagonal)


def assign(x, output=None):
    t = x if torch.is_tensor(x) else to_tensor(x)
    if output is None:
        return t.clone()
    output.copy_(t)
    return output


def clone(x, name=None):
    return x.clone()


# ------------------------------------------------------------------------ random
def seed(s):
    torch.manual_seed(s)
    np.random.seed(s % (2 ** 32))
    return torch.default_generator


def rand(shape, dtype=None, name=None):
    return torch.rand(_shape(shape), dtype=_dtype(dtype) or _default_dtype[0], device=_dev())


def randn(shape, dtype=None, name=None):
    return torch.randn(_shape(shape), dtype=_dtype(dtype) or _default_dtype[0], device=_dev())


standard_normal = randn


def randint(low=0, high=None, shape=(1,), dtype=None, name=None):
    if high is None:
        low, high = 0, low
    return torch.randint(low, high, _shape(shape), dtype=_dtype(dtype) or torch.int64, device=_dev())


def randint_like(x, low=0, high=None, dtype=None, name=None):
    if high is None:
        low, high = 0, low
    return torch.randint(low, high, x.shape, dtype=_dtype(dtype) or x.dtype, device=x.device)


def randperm(n, dtype="int64", name=None):
    return torch.randperm(n, dtype=_dtype(dtype), device=_dev())


def uniform(shape, dtype=None, min=-1.0, max=1.0, seed=0, name=None):
    return torch.empty(_shape(shape), dtype=_dtype(dtype) or _default_dtype[0], device=_dev()).uniform_(min, max)


def normal(mean=0.0, std=1.0, shape=None, name=None):
    if torch.is_tensor(mean) or torch.is_tensor(std):
        return torch.normal(mean, std)
    return torch.normal(mean, std, _shape(shape), device=_dev())


def bernoulli(x, name=None):
    return torch.bernoulli(x)


def multinomial(x, num_samples=1, replacement=False, name=None):
    return torch.multinomial(x, num_samples, replacement)


def poisson(x, name=None):
    return torch.poisson(x)


# -------------------------------------------------------------------------- math
def _ax(axis):
    if axis is None:
        return None
    if isinstance(axis, (list, tuple)):
        return tuple(axis)
    return axis


def add(x, y, name=None):
    return torch.add(x, y)


def subtract(x, y, name=None):
    return torch.sub(x, y)


def multiply(x, y, name=None):
    return torch.mul(x, y)


def divide(x, y, name=None):
    return torch.div(x, y)


def floor_divide(x, y, name=None):
    return torch.div(x, y, rounding_mode="floor")


def remainder(x, y, name=None):
    return torch.remainder(x, y)


mod = floor_mod = remainder


def pow(x, y, name=None):
    return torch.pow(x, y)


def scale(x, scale=1.0, bias=0.0, bias_after_scale=True, act=None, name=None):
    y = x * scale + bias if bias_after_scale else (x + bias) * scale
    return getattr(torch, act)(y) if act else y


def sum(x, axis=None, dtype=None, keepdim=False, name=None):
    a = _ax(axis)
    if a is None:
        return torch.sum(x, dtype=_dtype(dtype))
    return torch.sum(x, a, keepdim, dtype=_dtype(dtype))


def mean(x, axis=None, keepdim=False, name=None):
    a = _ax(axis)
    return torch.mean(x) if a is None else torch.mean(x, a, keepdim)


def max(x, axis=None, keepdim=False, name=None):
    a = _ax(axis)
    return torch.amax(x) if a is None else torch.amax(x, a, keepdim)


def min(x, axis=None, keepdim=False, name=None):
    a = _ax(axis)
    return torch.amin(x) if a is None else torch.amin(x, a, keepdim)


amax, amin = max, min


def prod(x, axis=None, keepdim=False, dtype=None, name=None):
    if axis is None:
        return torch.prod(x, dtype=_dtype(dtype))
    return torch.prod(x, axis, keepdim, dtype=_dtype(dtype))


def cumsum(x, axis=None, dtype=None, name=None):
    if axis is None:
        return torch.cumsum(x.reshape(-1), 0, dtype=_dtype(dtype))
    return torch.cumsum(x, axis, dtype=_dtype(dtype))


def cumprod(x, dim=None, dtype=None, name=None):
    return torch.cumprod(x, dim if dim is not None else 0, dtype=_dtype(dtype))


def logsumexp(x, axis=None, keepdim=False, name=None):
    a = _ax(axis)
    return torch.logsumexp(x, a if a is not None else tuple(range(x.dim())), keepdim)


def var(x, axis=None, unbiased=True, keepdim=False, name=None):
    a = _ax(axis)
    return torch.var(x, a, unbiased=unbiased, keepdim=keepdim)


def std(x, axis=None, unbiased=True, keepdim=False, name=None):
    a = _ax(axis)
    return torch.std(x, a, unbiased=unbiased, keepdim=keepdim)


def median(x, axis=None, keepdim=False, name=None):
    return torch.median(x) if axis is None else torch.median(x, axis, keepdim)[0]


def quantile(x, q, axis=None, keepdim=False, name=None):
    return torch.quantile(x, torch.as_tensor(q, dtype=x.dtype, device=x.device), axis, keepdim)


def all(x, axis=None, keepdim=False, name=None):
    return torch.all(x) if axis is None else torch.all(x, _ax(axis), keepdim)


def any(x, axis=None, keepdim=False, name=None):
    return torch.any(x) if axis is None else torch.any(x, _ax(axis), keepdim)


def matmul(x, y, transpose_x=False, transpose_y=False, name=None):
    if transpose_x:
        x = x.transpose(-1, -2)
    if transpose_y:
        y = y.transpose(-1, -2)
    return torch.matmul(x, y)


def bmm(x, y, name=None):
    return torch.bmm(x, y)


def mm(input, mat2, name=None):
    return torch.mm(input, mat2)


def dot(x, y, name=None):
    return (x * y).sum(-1)


def mv(x, vec, name=None):
    return torch.mv(x, vec)


def einsum(equation, *operands):
    return torch.einsum(equation, *operands)


def addmm(input, x, y, beta=1.0, alpha=1.0, name=None):
    return torch.addmm(input, x, y, beta=beta, alpha=alpha)


def inner(x, y, name=None):
    return torch.inner(x, y)


def outer(x, y, name=None):
    return torch.outer(x, y)


def cross(x, y, axis=9, name=None):
    return torch.cross(x, y, dim=-1 if axis == 9 else axis)


def kron(x, y, name=None):
    return torch.kron(x, y)


def clip(x, min=None, max=None, name=None):
    return torch.clamp(x, min, max)


def maximum(x, y, name=None):
    return torch.maximum(x, y)


def minimum(x, y, name=None):
    return torch.minimum(x, y)


def fmax(x, y, name=None):
    return torch.fmax(x, y)


def fmin(x, y, name=None):
    return torch.fmin(x, y)


def lerp(x, y, weight, name=None):
    return torch.lerp(x, y, weight)


def increment(x, value=1.0, name=None):
    return x.add_(value)


def nan_to_num(x, nan=0.0, posinf=None, neginf=None, name=None):
    return torch.nan_to_num(x, nan, posinf, neginf)


def logit(x, eps=None, name=None):
    return torch.logit(x, eps)


def trace(x, offset=0, axis1=0, axis2=1, name=None):
    return torch.diagonal(x, offset, axis1, axis2).sum(-1)


def diff(x, n=1, axis=-1, prepend=None, append=None, name=None):
    return torch.diff(x, n, axis, prepend, append)


def count_nonzero(x, axis=None, keepdim=False, name=None):
    r = torch.count_nonzero(x, _ax(axis))
    return r.unsqueeze(axis) if keepdim and axis is not None else r


def add_n(inputs, name=None):
    inputs = inputs if isinstance(inputs, (list, tuple)) else [inputs]
    out = inputs[0].clone()
    for t in inputs[1:]:
        out += t
    return out


def stanh(x, scale_a=0.67, scale_b=1.7159, name=None):
    return scale_b * torch.tanh(scale_a * x)


def _unary(fn):
    def f(x, name=None):
        return fn(x)

    f.__name__ = fn.__name__
    return f


for _n in ("exp", "log", "log2", "log10", "log1p", "sqrt", "rsqrt", "square", "abs", "sign", "sin", "cos", "tan",
           "asin", "acos", "atan", "sinh", "cosh", "tanh", "asinh", "acosh", "atanh", "ceil", "floor", "round",
           "trunc", "reciprocal", "erf", "erfinv", "isnan", "isinf", "isfinite", "neg", "expm1", "sigmoid",
           "digamma", "lgamma", "frac", "angle", "conj", "real", "imag"):
    globals()[_n] = _unary(getattr(torch, _n))


def atan2(x, y, name=None):
    return torch.atan2(x, y)


# ------------------------------------------------------------------ manipulation
def reshape(x, shape, name=None):
    return torch.reshape(x, _shape(shape))


def reshape_(x, shape, name=None):
    return x.view(_shape(shape))


def flatten(x, start_axis=0, stop_axis=-1, name=None):
    return torch.flatten(x, start_axis, stop_axis)


def squeeze(x, axis=None, name=None):
    if axis is None:
        return torch.squeeze(x)
    axes = [axis] if isinstance(axis, int) else list(axis)
    axes = [a % x.dim() for a in axes if x.shape[a] == 1]
    return torch.squeeze(x, tuple(axes)) if axes else x


def unsqueeze(x, axis, name=None):
    axes = [axis] if isinstance(axis, int) else sorted(a if a >= 0 else a + x.dim() + 1 for a in axis)
    for a in axes:
        x = torch.unsqueeze(x, a)
    return x


def transpose(x, perm, name=None):
    return x.permute(*perm)


def moveaxis(x, source, destination, name=None):
    return torch.movedim(x, source, destination)


def concat(x, axis=0, name=None):
    return torch.cat(list(x), int(axis))


def stack(x, axis=0, name=None):
    return torch.stack(list(x), axis)


def split(x, num_or_sections, axis=0, name=None):
    if isinstance(num_or_sections, int):
        return list(torch.chunk(x, num_or_sections, axis)) if x.shape[axis] % num_or_sections == 0 else \
            list(torch.split(x, math.ceil(x.shape[axis] / num_or_sections), axis))
    secs = list(num_or_sections)
    if -1 in secs:
        secs[secs.index(-1)] = x.shape[axis] - builtins.sum(s for s in secs if s != -1)
    return list(torch.split(x, secs, axis))


def chunk(x, chunks, axis=0, name=None):
    return list(torch.chunk(x, chunks, axis))


def unbind(input, axis=0):
    return list(torch.unbind(input, axis))


def unstack(x, axis=0, num=None):
    return list(torch.unbind(x, axis))


def gather(x, index, axis=None, name=None):
    return torch.index_select(x, axis or 0, index.reshape(-1).long())


def gather_nd(x, index, name=None):
    idx = index.long()
    k = idx.shape[-1]
    flat = idx.reshape(-1, k)
    out = x[tuple(flat[:, i] for i in range(k))]
    return out.reshape(*idx.shape[:-1], *x.shape[k:])


def scatter(x, index, updates, overwrite=True, name=None):
    out = x.clone()
    idx = index.reshape(-1).long()
    if overwrite:
        out[idx] = updates
    else:
        out[idx] = 0
        out.index_add_(0, idx, updates)
    return out


def scatter_nd_add(x, index, updates, name=None):
    out = x.clone()
    idx = index.long()
    k = idx.shape[-1]
    flat = idx.reshape(-1, k)
    out.index_put_(tuple(flat[:, i] for i in range(k)), updates.reshape(flat.shape[0], *x.shape[k:]),
                   accumulate=True)
    return out


def index_select(x, index, axis=0, name=None):
    return torch.index_select(x, axis, index.long())


def index_add(x, index, axis, value, name=None):
    return x.index_add(axis, index.long(), value)


def masked_select(x, mask, name=None):
    return torch.masked_select(x, mask)


def masked_fill(x, mask, value, name=None):
    return x.masked_fill(mask, value)


def where(condition, x=None, y=None, name=None):
    if x is None and y is None:
        return torch.nonzero(condition, as_tuple=True)
    return torch.where(condition, x, y)


def expand(x, shape, name=None):
    return x.expand(*_shape(shape))


def expand_as(x, y, name=None):
    return x.expand_as(y)


def broadcast_to(x, shape, name=None):
    return torch.broadcast_to(x, _shape(shape))


def broadcast_tensors(input, name=None):
    return list(torch.broadcast_tensors(*input))


def tile(x, repeat_times, name=None):
    return x.repeat(*_shape(repeat_times)) if len(_shape(repeat_times)) >= x.dim() else \
        torch.tile(x, tuple(_shape(repeat_times)))


def repeat_interleave(x, repeats, axis=None, name=None):
    return torch.repeat_interleave(x, repeats, axis)


def flip(x, axis, name=None):
    return torch.flip(x, [axis] if isinstance(axis, int) else list(axis))


def roll(x, shifts, axis=None, name=None):
    return torch.roll(x, shifts, axis)


def rot90(x, k=1, axes=(0, 1), name=None):
    return torch.rot90(x, k, axes)


def slice(input, axes, starts, ends):
    sl = [builtins.slice(None)] * input.dim()
    for a, s, e in zip(axes, starts, ends):
        sl[a] = builtins.slice(int(s), int(e))
    return input[tuple(sl)]


def strided_slice(x, axes, starts, ends, strides, name=None):
    sl = [builtins.slice(None)] * x.dim()
    for a, s, e, st in zip(axes, starts, ends, strides):
        sl[a] = builtins.slice(int(s), int(e), int(st))
    return x[tuple(sl)]


def cast(x, dtype):
    return x.to(_dtype(dtype))


def unique(x, return_index=False, return_inverse=False, return_counts=False, axis=None, dtype="int64", name=None):
    r = torch.unique(x, sorted=True, return_inverse=return_inverse, return_counts=return_counts, dim=axis)
    if not (return_index or return_inverse or return_counts):
        return r
    out = list(r) if isinstance(r, tuple) else [r]
    if return_index:
        u = out[0]
        first = torch.stack([(x.reshape(-1) == v).nonzero()[0, 0] for v in u.reshape(-1)]) if u.numel() else u.long()
        out.insert(1, first)
    return tuple(out)


def nonzero(x, as_tuple=False):
    return torch.nonzero(x, as_tuple=as_tuple)


def sort(x, axis=-1, descending=False, stable=False, name=None):
    return torch.sort(x, axis, descending, stable=stable)[0]


def argsort(x, axis=-1, descending=False, stable=False, name=None):
    return torch.sort(x, axis, descending, stable=stable)[1]


def argmax(x, axis=None, keepdim=False, dtype="int64", name=None):
    return torch.argmax(x, axis, keepdim).to(_dtype(dtype))


def argmin(x, axis=None, keepdim=False, dtype="int64", name=None):
    return torch.argmin(x, axis, keepdim).to(_dtype(dtype))


def topk(x, k, axis=-1, largest=True, sorted=True, name=None):
    r = torch.topk(x, int(k), axis, largest, sorted)
    return r.values, r.indices


def kthvalue(x, k, axis=-1, keepdim=False, name=None):
    r = torch.kthvalue(x, k, axis, keepdim)
    return r.values, r.indices


def mode(x, axis=-1, keepdim=False, name=None):
    r = torch.mode(x, axis, keepdim)
    return r.values, r.indices


def take_along_axis(arr, indices, axis, broadcast=True):
    return torch.take_along_dim(arr, indices.long(), axis)


def put_along_axis(arr, indices, values, axis, reduce="assign", include_self=True, broadcast=True):
    v = values if torch.is_tensor(values) else torch.full(indices.shape, values, dtype=arr.dtype,
                                                          device=arr.device)
    v = v.expand(indices.shape) if v.shape != indices.shape else v
    if reduce == "assign":
        return arr.scatter(axis, indices.long(), v)
    return arr.scatter_reduce(axis, indices.long(), v, {"add": "sum", "mul": "prod", "multiply": "prod"}.get(
        reduce, reduce), include_self=include_self)


def numel(x, name=None):
    return torch.tensor(x.numel(), dtype=torch.int64)


def shape(x):
    return torch.tensor(list(x.shape), dtype=torch.int64)


def rank(x):
    return x.dim()


def tolist(x):
    return x.tolist()


def searchsorted(sorted_sequence, values, out_int32=False, right=False, name=None):
    return torch.searchsorted(sorted_sequence, values, out_int32=out_int32, right=right)


def bucketize(x, sorted_sequence, out_int32=False, right=False, name=None):
    return torch.bucketize(x, sorted_sequence, out_int32=out_int32, right=right)


def histogram(input, bins=100, min=0, max=0, name=None):
    if min == max == 0:
        min, max = float(input.min()), float(input.max())
    return torch.histc(input.float(), bins, min, max).long()


# ------------------------------------------------------------------------- logic
def _bin(fn):
    def f(x, y, name=None):
        return fn(x, y)

    return f


equal = _bin(torch.eq)
not_equal = _bin(torch.ne)
less_than = _bin(torch.lt)
less_equal = _bin(torch.le)
greater_than = _bin(torch.gt)
greater_equal = _bin(torch.ge)
logical_and = _bin(torch.logical_and)
logical_or = _bin(torch.logical_or)
logical_xor = _bin(torch.logical_xor)
bitwise_and = _bin(torch.bitwise_and)
bitwise_or = _bin(torch.bitwise_or)
bitwise_xor = _bin(torch.bitwise_xor)


def logical_not(x, name=None):
    return torch.logical_not(x)


def bitwise_not(x, name=None):
    return torch.bitwise_not(x)


def equal_all(x, y, name=None):
    return torch.tensor(bool(torch.equal(x, y)))


def allclose(x, y, rtol=1e-05, atol=1e-08, equal_nan=False, name=None):
    return torch.tensor(bool(torch.allclose(x, y, rtol, atol, equal_nan)))


def isclose(x, y, rtol=1e-05, atol=1e-08, equal_nan=False, name=None):
    return torch.isclose(x, y, rtol, atol, equal_nan)


def is_tensor(x):
    return torch.is_tensor(x)


def is_floating_point(x):
    return x.is_floating_point()


def is_empty(x, name=None):
    return torch.tensor(x.numel() == 0)


# ------------------------------------------------------------------------ linalg
class linalg:
    @staticmethod
    def norm(x, p="fro", axis=None, keepdim=False, name=None):
        if p == "fro" and axis is None:
            return torch.linalg.norm(x.reshape(-1), 2)
        return torch.linalg.norm(x, p if p != "fro" else None, _ax(axis), keepdim) if axis is not None else \
            torch.linalg.norm(x.reshape(-1), p)

    inv = staticmethod(lambda x, name=None: torch.linalg.inv(x))
    det = staticmethod(lambda x, name=None: torch.linalg.det(x))
    slogdet = staticmethod(lambda x, name=None: torch.stack(torch.linalg.slogdet(x)))
    svd = staticmethod(lambda x, full_matrices=False, name=None: torch.linalg.svd(x, full_matrices))
    qr = staticmethod(lambda x, mode="reduced", name=None: torch.linalg.qr(x, mode))
    eig = staticmethod(lambda x, name=None: torch.linalg.eig(x))
    eigh = staticmethod(lambda x, UPLO="L", name=None: torch.linalg.eigh(x, UPLO))
    eigvals = staticmethod(lambda x, name=None: torch.linalg.eigvals(x))
    eigvalsh = staticmethod(lambda x, UPLO="L", name=None: torch.linalg.eigvalsh(x, UPLO))
    cholesky = staticmethod(lambda x, upper=False, name=None: torch.linalg.cholesky(x, upper=upper))
    solve = staticmethod(lambda x, y, name=None: torch.linalg.solve(x, y))
    matrix_power = staticmethod(lambda x, n, name=None: torch.linalg.matrix_power(x, n))
    pinv = staticmethod(lambda x, rcond=1e-15, hermitian=False, name=None: torch.linalg.pinv(x, rtol=rcond,
                                                                                              hermitian=hermitian))
    matrix_rank = staticmethod(lambda x, tol=None, hermitian=False, name=None: torch.linalg.matrix_rank(
        x, atol=tol, hermitian=hermitian))
    cond = staticmethod(lambda x, p=None, name=None: torch.linalg.cond(x, p))
    lstsq = staticmethod(lambda x, y, rcond=None, driver=None, name=None: torch.linalg.lstsq(x, y, rcond))
    multi_dot = staticmethod(lambda x, name=None: torch.linalg.multi_dot(x))
    cross = staticmethod(lambda x, y, axis=-1, name=None: torch.linalg.cross(x, y, dim=axis))


def norm(x, p="fro", axis=None, keepdim=False, name=None):
    return linalg.norm(x, p, axis, keepdim)


def t(x, name=None):
    return x.t() if x.dim() == 2 else x


no_grad = _eager.no_grad
enable_grad = _eager.enable_grad
set_grad_enabled = _eager.set_grad_enabled
is_grad_enabled = _eager.is_grad_enabled


def grad(outputs, inputs, grad_outputs=None, retain_graph=None, create_graph=False, only_inputs=True,
         allow_unused=False, no_grad_vars=None):
    """``paddle.grad`` on the framework engine (raw torch tensors: torch autograd)."""
    outs = outputs if isinstance(outputs, (list, tuple)) else [outputs]
    ins = inputs if isinstance(inputs, (list, tuple)) else [inputs]
    if builtins.any(isinstance(t, Tensor) for t in list(outs) + list(ins)):
        r = _eager.grad(list(outs), list(ins), grad_outputs, retain_graph, create_graph, allow_unused)
        return r if isinstance(r, list) else [r]
    return list(torch.autograd.grad(outs, ins, grad_outputs, retain_graph, create_graph, allow_unused=allow_unused))


# --------------------------------------------------------- Tensor method patches
def _wrap_module_functions():
    import types

    g = globals()
    for name, fn in list(g.items()):
        if name.startswith("_") or not isinstance(fn, types.FunctionType) or fn.__module__ != __name__:
            continue
        if name in ("no_grad", "enable_grad", "set_grad_enabled", "is_grad_enabled",
                    "set_default_dtype", "get_default_dtype", "set_device", "get_device", "seed", "grad"):
            continue
        g[name] = _eager.wraps_outputs(fn)


_wrap_module_functions()
