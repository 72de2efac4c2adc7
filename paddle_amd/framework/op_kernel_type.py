"""Typed kernel dispatch and input data transforms (SURVEY §2.1 #5 operator runtime,
#13 data transform).

Reference: ``OperatorWithKernel::RunImpl`` (framework/operator.cc:657-730) picks a
kernel by ``GetExpectedKernelType`` (``IndicateDataType`` + the context place,
operator.cc:797-833) out of the op's ``OpKernelMap`` keyed by ``OpKernelType``
(op_kernel_type.h: place, data type, layout, library), then ``TryTransferData``
(operator.cc:743-795) converts every input whose own kernel type differs, into a
transfer scope, with ``TransformData`` (data_transform.cc:33-90: layout, then data
type, then device).

Here an op may register several kernels with :func:`register_op_kernel`, e.g. a
PLAIN kernel for any place and a NATIVE (hand-written HIP) kernel for the GPU that
only covers fp32; :func:`select` chooses one for the expected key and
:func:`prepare_inputs` hands the kernel transformed copies of the inputs (the
scope's variables are left untouched, as with the reference's transfer scope).
Ops without typed kernels keep their single place-agnostic kernel.

Dtype fallback: when no kernel is registered for the expected data type but one at
the same place / library is, the inputs are cast to that kernel's first data type
(the reference throws there; later Paddle versions fall back the same way).  With
no typed kernel for the place at all, the op's place-agnostic kernel runs on the
inputs as they are.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from . import core


class DataLayout:
    ANY = "AnyLayout"
    NCHW = "NCHW"
    NHWC = "NHWC"


class LibraryType:
    PLAIN = "PLAIN"    # torch / host code, any place
    NATIVE = "NATIVE"  # hand-written gfx950 kernels (csrc/kernels)


@dataclass(frozen=True)
class OpKernelType:
    place: str                       # "CPU" | "GPU"
    dtype: torch.dtype | None
    layout: str = DataLayout.ANY
    library: str = LibraryType.PLAIN

    def __str__(self):
        return f"data_type[{self.dtype}]:data_layout[{self.layout}]:place[{self.place}]:library_type[{self.library}]"


def place_kind(place_or_device) -> str:
    if isinstance(place_or_device, torch.device):
        return "GPU" if place_or_device.type == "cuda" else "CPU"
    return "GPU" if place_or_device.torch_device().type == "cuda" else "CPU"


def register_op_kernel(op_type, place, dtypes, layout=DataLayout.ANY, library=LibraryType.PLAIN):
    """Register ``fn(ctx)`` for ``op_type`` under every (place, dtype) of ``dtypes``."""
    from . import registry as R

    def deco(fn):
        info = R.OP_REGISTRY.get(op_type)
        if info is None:
            raise KeyError(f"op {op_type} not declared")
        if info.kernels is None:
            info.kernels = {}
        for dt in dtypes:
            info.kernels[OpKernelType(place, dt, layout, library)] = fn
        return fn

    return deco


def indicate_data_type(ctx):
    """dtype of the first initialised floating tensor input (operator.cc:797)."""
    for vals in ctx.ins.values():
        for v in vals or []:
            t = v.tensor if isinstance(v, core.LoDTensor) else (
                v.get_tensor().tensor if isinstance(v, core.SelectedRows) else v)
            if isinstance(t, torch.Tensor) and t.is_floating_point():
                return t.dtype
    return torch.float32


def expected_kernel_type(info, ctx) -> OpKernelType:
    if info.expected_kernel_type is not None:
        return info.expected_kernel_type(ctx)
    layout = ctx.attr("data_format", ctx.attr("data_layout", DataLayout.ANY))
    if layout not in (DataLayout.NCHW, DataLayout.NHWC):
        layout = DataLayout.ANY
    place = place_kind(ctx.place)
    lib = LibraryType.NATIVE if place == "GPU" and any(
        k.library == LibraryType.NATIVE and k.place == "GPU" for k in info.kernels) else LibraryType.PLAIN
    return OpKernelType(place, indicate_data_type(ctx), layout, lib)


def select(info, key: OpKernelType):
    """(kernel, kernel type) for ``key``: exact, then any layout, then dtype fallback,
    then the PLAIN library (a NATIVE key with no match)."""
    ks = info.kernels
    cands = [key, OpKernelType(key.place, key.dtype, DataLayout.ANY, key.library)]
    for k in cands:
        if k in ks:
            return ks[k], k
    for lib in (key.library, LibraryType.PLAIN):
        same = [k for k in ks if k.place == key.place and k.library == lib]
        for k in same:
            if k.dtype == key.dtype:
                return ks[k], k
        if same:
            return ks[same[0]], same[0]
    if info.kernel is not None:
        return info.kernel, None  # the place-agnostic kernel: inputs as they are
    raise NotImplementedError(f"op {info.type} does not have kernel for {key}")


def kernel_type_for_var(t: torch.Tensor, layout=DataLayout.ANY) -> OpKernelType:
    return OpKernelType(place_kind(t.device), t.dtype, layout)


def need_transform(var_t: OpKernelType, exp_t: OpKernelType) -> bool:
    if var_t.place != exp_t.place:
        return True
    if exp_t.dtype is not None and var_t.dtype != exp_t.dtype and var_t.dtype is not None \
            and var_t.dtype.is_floating_point and exp_t.dtype.is_floating_point:
        return True
    return var_t.layout != DataLayout.ANY and exp_t.layout != DataLayout.ANY and var_t.layout != exp_t.layout


def transform_data(exp_t: OpKernelType, var_t: OpKernelType, t: torch.Tensor) -> torch.Tensor:
    """Layout, then data type, then device (data_transform.cc:33-90)."""
    if var_t.layout != DataLayout.ANY and exp_t.layout != DataLayout.ANY and var_t.layout != exp_t.layout \
            and t.dim() == 4:
        perm = (0, 2, 3, 1) if exp_t.layout == DataLayout.NHWC else (0, 3, 1, 2)
        t = t.permute(*perm).contiguous()
    if exp_t.dtype is not None and t.is_floating_point() and exp_t.dtype.is_floating_point and t.dtype != exp_t.dtype:
        t = t.to(exp_t.dtype)
    dev_kind = place_kind(t.device)
    if dev_kind != exp_t.place:
        t = t.to("cuda" if exp_t.place == "GPU" else "cpu")
    return t


def prepare_inputs(info, ctx, ktype: OpKernelType):
    """Replace ``ctx.ins`` values with transformed copies where the kernel needs them
    (the transfer scope of operator.cc:743).  Slots listed in ``info.host_slots``
    stay where they are (host-side shape / length inputs)."""
    host = info.host_slots or ()
    for slot, vals in ctx.ins.items():
        if slot in host or not vals:
            continue
        new = None
        for i, v in enumerate(vals):
            if isinstance(v, core.LoDTensor) and isinstance(v.tensor, torch.Tensor):
                t = v.tensor
                var_t = kernel_type_for_var(t, getattr(v, "layout", DataLayout.ANY))
                if not t.is_floating_point():
                    var_t = OpKernelType(var_t.place, None, var_t.layout)
                if need_transform(var_t, ktype):
                    if new is None:
                        new = list(vals)
                    lay = ktype.layout if var_t.layout != DataLayout.ANY and ktype.layout != DataLayout.ANY \
                        else v.layout
                    new[i] = core.LoDTensor(transform_data(ktype, var_t, t), v.lod(), lay)
        if new is not None:
            ctx.ins[slot] = new
