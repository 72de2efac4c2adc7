"""Operator registry, kernel execution context, grad-op makers, shape inference.

Parity: ``REGISTER_OPERATOR`` / ``OpProtoAndCheckerMaker`` /
``OpInfoMap`` (framework/op_registry.h:38-287, op_proto_maker.h:38, op_info.h:68),
``OperatorWithKernel::RunImpl`` dispatch (operator.cc:657), compile-time
``InferShape`` (op_desc.cc:469) and ``DefaultGradOpDescMaker``
(grad_op_desc_maker.h:156) exposed to Python as ``get_grad_op_desc``.

Design: an op is registered once with a compact I/O spec and ONE kernel function
``kernel(ctx)`` written against :class:`KernelContext`; the kernel receives
torch tensors that live on the op's place (CPU or the HIP device) and calls
either PyTorch-ROCm or the hand-written gfx950 kernels.  Because kernels are
pure functions of their context, the same code serves four purposes:
  * runtime execution (Executor),
  * compile-time shape inference (run on ``meta`` tensors -- no per-op
    InferShape boilerplate unless an op is data-dependent),
  * automatic gradient kernels for ops without a hand-written ``*_grad``
    kernel (vector-Jacobian product of the forward kernel via autograd),
  * the OpTest harness (tests call kernels directly on numpy inputs).
Slot spec syntax: ``"X"`` plain, ``"X*"`` duplicable, ``"X?"`` dispensable,
``"X~"`` intermediate; combinations allowed (``"X*?"``).
"""
from __future__ import annotations

import copy
import weakref
from dataclasses import dataclass, field

import torch

from ..autograd import engine as _eager
from . import core
from .proto import AttrType

GRAD_SUFFIX = "@GRAD"
EMPTY_VAR = "@EMPTY@"
TEMP_VAR = "@TEMP@"


def grad_var_name(name: str) -> str:
    return name + GRAD_SUFFIX


class OpRole:
    """framework/op_proto_maker.h:25-41."""
    Forward = 0x0000
    Backward = 0x0001
    Optimize = 0x0002
    RPC = 0x0003
    Loss = 0x0100
    LRSched = 0x0010


OP_ROLE_ATTR = "op_role"
OP_ROLE_VAR_ATTR = "op_role_var"


@dataclass
class Slot:
    name: str
    duplicable: bool = False
    dispensable: bool = False
    intermediate: bool = False
    comment: str = ""

    @staticmethod
    def parse(spec: str) -> "Slot":
        n = spec.rstrip("*?~")
        flags = spec[len(n):]
        return Slot(n, "*" in flags, "?" in flags, "~" in flags)


@dataclass
class OpInfo:
    type: str
    inputs: list
    outputs: list
    attrs: dict  # name -> default
    kernel: callable = None
    infer_shape: callable = None
    grad_maker: object = "default"  # "default" | None | callable(op, no_grad_set) -> list[dict]
    grad_of: str | None = None  # for *_grad ops built by the default maker
    comment: str = ""
    no_infer: bool = False  # skip compile-time meta inference (side-effecting ops)
    share_lod: bool = True
    # typed kernels (op_kernel_type.register_op_kernel): OpKernelType -> fn; None = the
    # single place-agnostic ``kernel``
    kernels: dict | None = None
    expected_kernel_type: callable = None  # ctx -> OpKernelType (GetExpectedKernelType override)
    host_slots: tuple | None = None  # input slots the data transform leaves in place

    def input_names(self):
        return [s.name for s in self.inputs]

    def output_names(self):
        return [s.name for s in self.outputs]

    def slot(self, name, out=False):
        for s in (self.outputs if out else self.inputs):
            if s.name == name:
                return s
        return None


OP_REGISTRY: "dict[str, OpInfo]" = {}


def register_op(type, inputs=(), outputs=(), attrs=None, grad="default", infer_shape=None, comment="",
                no_infer=False, share_lod=True):
    """Decorator registering ``kernel(ctx)`` for op ``type``."""

    def deco(fn):
        info = OpInfo(type, [Slot.parse(s) for s in inputs], [Slot.parse(s) for s in outputs],
                      dict(attrs or {}), fn, infer_shape, grad, None, comment or (fn.__doc__ or ""),
                      no_infer, share_lod)
        OP_REGISTRY[type] = info
        return fn

    return deco


def register_kernel(type):
    """Attach/override the kernel of an already-declared op (e.g. a hand-written ``*_grad``)."""

    def deco(fn):
        info = OP_REGISTRY.get(type)
        if info is None:
            raise KeyError(f"op {type} not declared")
        info.kernel = fn
        return fn

    return deco


def get_op_info(type) -> OpInfo:
    info = OP_REGISTRY.get(type)
    if info is None and type.endswith("_grad") and type[:-5] in OP_REGISTRY:
        info = _make_auto_grad_info(type[:-5])
    if info is None:
        raise KeyError(f"Operator '{type}' is not registered in paddle_amd")
    return info


def has_op(type):
    try:
        get_op_info(type)
        return True
    except KeyError:
        return False


# ---------------------------------------------------------------- kernel context


class KernelContext:
    """What a kernel sees: inputs (runtime values) by slot, attrs, place; collects outputs."""

    __slots__ = ("type", "ins", "out_names", "attrs", "place", "device", "results", "scope", "op",
                 "executor", "meta")

    def __init__(self, type, ins, out_names, attrs, place=None, scope=None, op=None, executor=None, meta=False):
        self.type = type
        self.ins = ins  # slot -> list of runtime values (LoDTensor/SelectedRows/...), None for missing
        self.out_names = out_names  # slot -> list of var names
        self.attrs = attrs
        self.place = place or core.CPUPlace()
        self.device = self.place.torch_device() if not meta else torch.device("meta")
        self.results = {}
        self.scope = scope
        self.op = op
        self.executor = executor
        self.meta = meta

    # ---- inputs
    def has_input(self, slot):
        v = self.ins.get(slot)
        return bool(v) and v[0] is not None

    def input_value(self, slot, i=0):
        v = self.ins.get(slot)
        if not v or i >= len(v):
            return None
        return v[i]

    def input(self, slot, i=0):
        v = self.input_value(slot, i)
        if v is None:
            return None
        if isinstance(v, core.LoDTensor):
            return v.tensor
        if isinstance(v, core.SelectedRows):
            return v.get_tensor().tensor
        return v

    def inputs(self, slot):
        out = []
        for v in self.ins.get(slot, []) or []:
            if isinstance(v, core.LoDTensor):
                out.append(v.tensor)
            elif isinstance(v, core.SelectedRows):
                out.append(v.get_tensor().tensor)
            else:
                out.append(v)
        return out

    def input_values(self, slot):
        return list(self.ins.get(slot, []) or [])

    def input_lod(self, slot, i=0):
        v = self.input_value(slot, i)
        return v.lod() if isinstance(v, core.LoDTensor) else []

    def num_inputs(self, slot):
        return len(self.ins.get(slot, []) or [])

    def attr(self, name, default=None):
        return self.attrs.get(name, default)

    # ---- outputs
    def has_output(self, slot):
        n = self.out_names.get(slot)
        return bool(n) and n[0] != EMPTY_VAR

    def output_names(self, slot):
        return list(self.out_names.get(slot, []))

    def set_output(self, slot, tensor, lod=None, i=0):
        lst = self.results.setdefault(slot, [])
        while len(lst) <= i:
            lst.append(None)
        if isinstance(tensor, (core.LoDTensor, core.SelectedRows, core.LoDTensorArray)) or not isinstance(
                tensor, torch.Tensor):
            lst[i] = tensor
        else:
            lst[i] = core.LoDTensor(tensor, lod)

    def set_outputs(self, slot, tensors, lods=None):
        for i, t in enumerate(tensors):
            self.set_output(slot, t, lods[i] if lods else None, i)

    # ---- helpers
    def zeros(self, shape, dtype=torch.float32):
        return torch.zeros(shape, dtype=dtype, device=self.device)

    def float_dtype(self):
        return torch.float32


def call_kernel(info: OpInfo, ctx: KernelContext):
    """OperatorWithKernel::RunImpl: typed kernel selection + input data transform
    (op_kernel_type.py) when the op registered typed kernels, else its one kernel.
    Shape inference on meta tensors always runs the place-agnostic kernel."""
    if info.kernels and not ctx.meta:
        from . import op_kernel_type as K

        fn, kt = K.select(info, K.expected_kernel_type(info, ctx))
        if kt is not None:
            K.prepare_inputs(info, ctx, kt)
        fn(ctx)
    else:
        info.kernel(ctx)


def run_kernel(info: OpInfo, ctx: KernelContext):
    call_kernel(info, ctx)
    if info.share_lod:
        _default_share_lod(info, ctx)
    return ctx.results


def _default_share_lod(info, ctx):
    first = None
    for s in info.inputs:
        v = ctx.input_value(s.name)
        if isinstance(v, core.LoDTensor) and v.lod():
            first = v
            break
    if first is None or first.tensor is None:
        return
    rows = first.tensor.shape[0] if first.tensor.dim() else None
    for slot, vals in ctx.results.items():
        for v in vals:
            if isinstance(v, core.LoDTensor) and not v.lod() and v.tensor is not None and v.tensor.dim() \
                    and v.tensor.shape[0] == rows:
                v.set_lod(first.lod())


# ---------------------------------------------------------------- grad op makers


def default_grad_op_descs(op, no_grad_set=frozenset()):
    """DefaultGradOpDescMaker: X_grad takes all inputs, outputs, Out@GRAD; emits In@GRAD."""
    info = get_op_info(op.type)
    g_inputs, g_outputs = {}, {}
    for s in info.inputs:
        g_inputs[s.name] = list(op.input(s.name))
    for s in info.outputs:
        g_inputs[s.name] = list(op.output(s.name))
        g_inputs[s.name + GRAD_SUFFIX] = [grad_var_name(n) for n in op.output(s.name)]
    for s in info.inputs:
        names = []
        for n in op.input(s.name):
            names.append(EMPTY_VAR if n in no_grad_set else grad_var_name(n))
        g_outputs[s.name + GRAD_SUFFIX] = names
    return [dict(type=op.type + "_grad", inputs=g_inputs, outputs=g_outputs, attrs=dict(op.all_attrs()))]


def make_grad_op_descs(op, no_grad_set=frozenset(), sub_blocks=None):
    info = get_op_info(op.type)
    if info.grad_maker is None:
        return []
    if info.grad_maker == "default":
        return default_grad_op_descs(op, no_grad_set)
    return info.grad_maker(op, no_grad_set)


# ---------------------------------------------------------------- automatic grad kernels

_AUTO_GRAD: dict = {}


def _make_auto_grad_info(fwd_type):
    if fwd_type in _AUTO_GRAD:
        return _AUTO_GRAD[fwd_type]
    fwd = OP_REGISTRY[fwd_type]
    ins = [Slot(s.name, s.duplicable, True) for s in fwd.inputs]
    ins += [Slot(s.name, s.duplicable, True) for s in fwd.outputs]
    ins += [Slot(s.name + GRAD_SUFFIX, s.duplicable, True) for s in fwd.outputs]
    outs = [Slot(s.name + GRAD_SUFFIX, s.duplicable, True) for s in fwd.inputs]
    info = OpInfo(fwd_type + "_grad", ins, outs, dict(fwd.attrs), None, None, None, fwd_type,
                  f"auto VJP of {fwd_type}", True, False)
    info.kernel = lambda ctx, _f=fwd: auto_grad_kernel(_f, ctx)
    _AUTO_GRAD[fwd_type] = info
    OP_REGISTRY[info.type] = info
    return info


# Forward graphs kept for the auto-VJP grad ops of a training program: the forward
# op runs once under autograd (BlockExecutor marks the ops whose grads are auto
# and present in the program) and its grad op takes the VJP of the stashed graph
# instead of re-running the forward kernel.  Keyed by id() of every output tensor (with a
# weak reference that must still resolve to that same tensor)
# the forward op stored in the scope; cleared at the start of every top-level run.
_STASH: dict = {}


def clear_stash():
    _STASH.clear()


def is_auto_grad(grad_type):
    """True when ``grad_type`` is served by auto_grad_kernel (not a hand-written grad)."""
    if not grad_type.endswith("_grad"):
        return False
    try:
        info = get_op_info(grad_type)
    except Exception:  # noqa: BLE001
        return False
    return _AUTO_GRAD.get(grad_type[:-5]) is info


def run_kernel_stash(info: OpInfo, ctx: KernelContext):
    """Run a forward kernel with its float inputs as autograd leaves, keep the
    graph for the grad op, hand detached outputs to the scope."""
    op = ctx.op
    inplace = set()
    if op is not None:
        outs_names = {n for names in op.outputs.values() for n in names}
        inplace = {n for names in op.inputs.values() for n in names if n in outs_names}
    leaves = {}
    for s in info.inputs:
        vals = ctx.ins.get(s.name) or []
        names = op.input(s.name) if op is not None else []
        new = []
        for i, v in enumerate(vals):
            n = names[i] if i < len(names) else None
            if isinstance(v, core.LoDTensor) and v.tensor is not None and v.tensor.is_floating_point() \
                    and n not in inplace:
                t = _eager.to_tensor_handle(v.tensor.detach(), stop_gradient=False)
                leaves[(s.name, i)] = t
                new.append(core.LoDTensor(t, v.lod()))
            else:
                new.append(v)
        ctx.ins[s.name] = new
    with torch.enable_grad(), _eager.enable_grad():
        call_kernel(info, ctx)
    if info.share_lod:
        _default_share_lod(info, ctx)
    graph_outs = {}
    for slot, vals in ctx.results.items():
        for i, r in enumerate(vals):
            rt = r.tensor if isinstance(r, core.LoDTensor) else r
            if isinstance(rt, torch.Tensor) and _eager.tracked(rt):
                graph_outs[(slot, i)] = rt
                d = _eager._raw(rt).detach()
                vals[i] = core.LoDTensor(d, r.lod()) if isinstance(r, core.LoDTensor) else d
    if graph_outs and leaves:
        entry = (leaves, graph_outs)
        for (slot, i) in graph_outs:
            r = ctx.results[slot][i]
            t = r.tensor if isinstance(r, core.LoDTensor) else r
            # keyed by id, validated by identity: an id recycled after the output
            # object died never picks up another op's graph
            _STASH[id(t)] = (weakref.ref(t), entry)
    return ctx.results


def _stashed_vjp(fwd: OpInfo, ctx: KernelContext):
    entry = None
    for s in fwd.outputs:
        for v in ctx.input_values(s.name):
            t = v.tensor if isinstance(v, core.LoDTensor) else v
            if isinstance(t, torch.Tensor) and id(t) in _STASH:
                ref, e = _STASH[id(t)]
                if ref() is t:
                    entry = e
                    break
                _STASH.pop(id(t), None)  # a recycled id: the stashed forward is gone
        if entry is not None:
            break
    if entry is None:
        return None
    leaves, graph_outs = entry
    for (slot, i), rt in graph_outs.items():
        vals = ctx.input_values(slot)
        if i < len(vals):
            t = vals[i].tensor if isinstance(vals[i], core.LoDTensor) else vals[i]
            _STASH.pop(id(t), None)
    outs, gouts = [], []
    for (slot, i), rt in graph_outs.items():
        gvals = ctx.input_values(slot + GRAD_SUFFIX)
        if i >= len(gvals) or gvals[i] is None:
            continue
        gt = gvals[i].tensor if isinstance(gvals[i], core.LoDTensor) else gvals[i]
        if gt is None:
            continue
        outs.append(rt)
        gouts.append(gt.to(rt.dtype).reshape(rt.shape))
    keys = list(leaves.keys())
    grads = _engine_vjp(outs, [leaves[k] for k in keys], gouts)
    return dict(zip(keys, grads))


def _engine_vjp(outs, leaves, gouts):
    """VJP on the framework's eager engine (explicit per-op backward rules and the
    fused ops' own backward kernels; autograd/engine.py) -- not torch autograd."""
    if not outs or not leaves:
        return [None] * len(leaves)
    r = _eager.grad(outs, leaves, [_eager._raw(g) for g in gouts], retain_graph=False, allow_unused=True)
    r = r if isinstance(r, list) else [r]
    return [None if g is None else _eager._raw(g) for g in r]


def auto_grad_kernel(fwd: OpInfo, ctx: KernelContext):
    """Gradient of any registered forward kernel: the VJP of the forward graph the
    executor stashed, or else re-run the forward under autograd on leaf copies of
    the float inputs and take the vector-Jacobian product with the incoming output
    gradients (replaces per-op GradOpMaker + grad kernel pairs)."""
    gmap = _stashed_vjp(fwd, ctx)
    if gmap is not None:
        _write_input_grads(fwd, ctx, gmap)
        return
    leaves = {}
    fins = {}
    for s in fwd.inputs:
        vals = []
        for i, v in enumerate(ctx.input_values(s.name)):
            if isinstance(v, core.LoDTensor) and v.tensor is not None and v.tensor.is_floating_point():
                t = _eager.to_tensor_handle(v.tensor.detach(), stop_gradient=False)
                leaves[(s.name, i)] = t
                vals.append(core.LoDTensor(t, v.lod()))
            else:
                vals.append(v)
        fins[s.name] = vals
    fctx = KernelContext(fwd.type, fins, {s.name: [f"{s.name}#{k}" for k in range(max(1, len(ctx.input_values(s.name))))]
                                          for s in fwd.outputs}, ctx.attrs, ctx.place)
    with torch.enable_grad(), _eager.enable_grad():
        call_kernel(fwd, fctx)
    outs, gouts = [], []
    for s in fwd.outputs:
        gvals = ctx.input_values(s.name + GRAD_SUFFIX)
        res = fctx.results.get(s.name, [])
        for i, r in enumerate(res):
            if r is None or i >= len(gvals) or gvals[i] is None:
                continue
            rt = r.tensor if isinstance(r, core.LoDTensor) else r
            g = gvals[i]
            gt = g.tensor if isinstance(g, core.LoDTensor) else g
            if gt is None or not isinstance(rt, torch.Tensor) or not _eager.tracked(rt):
                continue
            outs.append(rt)
            gouts.append(gt.to(rt.dtype).reshape(rt.shape))
    keys = list(leaves.keys())
    grads = _engine_vjp(outs, [leaves[k] for k in keys], gouts)
    _write_input_grads(fwd, ctx, dict(zip(keys, grads)))


def _write_input_grads(fwd, ctx, gmap):
    for s in fwd.inputs:
        slot = s.name + GRAD_SUFFIX
        if not ctx.has_output(slot):
            continue
        for i, v in enumerate(ctx.input_values(s.name)):
            g = gmap.get((s.name, i))
            if g is None:
                src = v.tensor if isinstance(v, core.LoDTensor) else None
                if src is None:
                    continue
                g = torch.zeros_like(src)
            ctx.set_output(slot, _eager._raw(g).detach(), v.lod() if isinstance(v, core.LoDTensor) else None, i)


# ---------------------------------------------------------------- compile-time shape inference

SENTINEL = 8191  # stands in for -1 (unknown) dims during meta execution


def infer_shapes_meta(info: OpInfo, in_descs, out_names, attrs):
    """Run the kernel on meta tensors. in_descs: slot -> list of (shape, dtype_vt, lod_level) or None.
    Returns slot -> list of (shape, dtype_vt) (or None when inference is impossible)."""
    ins = {}
    for slot, lst in in_descs.items():
        vals = []
        for d in lst:
            if d is None:
                vals.append(None)
                continue
            shape, vt, lod_level = d
            shp = [SENTINEL if (s is None or s < 0) else int(s) for s in shape]
            t = torch.empty(shp, dtype=core.to_torch_dtype(vt), device="meta")
            lod = [[0, shp[0]]] * lod_level if (lod_level and shp) else []
            vals.append(core.LoDTensor(t, lod))
        ins[slot] = vals
    ctx = KernelContext(info.type, ins, out_names, attrs, core.CPUPlace(), meta=True)
    info.kernel(ctx)
    out = {}
    for slot, vals in ctx.results.items():
        lst = []
        for v in vals:
            t = v.tensor if isinstance(v, core.LoDTensor) else (v if isinstance(v, torch.Tensor) else None)
            if t is None:
                lst.append(None)
                continue
            shape = [-1 if (s % SENTINEL == 0 and s > 0) else int(s) for s in t.shape]
            lst.append((shape, core.convert_dtype(t.dtype)))
        out[slot] = lst
    return out


def attr_type_of(v):
    if isinstance(v, bool):
        return AttrType.BOOLEAN
    if isinstance(v, int):
        return AttrType.INT if -2**31 <= v < 2**31 else AttrType.LONG
    if isinstance(v, float):
        return AttrType.FLOAT
    if isinstance(v, str):
        return AttrType.STRING
    if isinstance(v, (list, tuple)):
        if not v:
            return AttrType.INTS
        if all(isinstance(x, bool) for x in v):
            return AttrType.BOOLEANS
        if all(isinstance(x, int) for x in v):
            return AttrType.INTS
        if all(isinstance(x, (int, float)) for x in v):
            return AttrType.FLOATS
        if all(isinstance(x, str) for x in v):
            return AttrType.STRINGS
    return AttrType.STRING


def get_all_op_protos():
    """OpProto messages for every registered op (pybind.cc:358 get_all_op_protos)."""
    from .proto import OpProtoPB

    out = []
    for t, info in sorted(OP_REGISTRY.items()):
        p = OpProtoPB(type=t, comment=info.comment or t)
        for s in info.inputs:
            p.inputs.add(name=s.name, comment=s.comment or s.name, duplicable=s.duplicable,
                         dispensable=s.dispensable, intermediate=s.intermediate)
        for s in info.outputs:
            p.outputs.add(name=s.name, comment=s.comment or s.name, duplicable=s.duplicable,
                          dispensable=s.dispensable, intermediate=s.intermediate)
        for a, d in info.attrs.items():
            p.attrs.add(name=a, type=attr_type_of(d), comment=a)
        out.append(p)
    return out


def clone_attrs(a):
    return copy.deepcopy(a)
