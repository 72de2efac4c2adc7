"""paddle.fluid.framework: Program / Block / Operator / Variable / Parameter.

Parity: python/paddle/fluid/framework.py (Variable :207, Operator :496, Block :923,
Program :1407, Parameter :1942, default programs / program_guard / name_scope
:2026-2094).  Operator construction validates slots and attributes against the op
registry and runs compile-time InferVarType/InferShape (framework.py:656-659); the
shape inference here executes the op's kernel on ``meta`` tensors.

The IR is kept as plain Python objects; ``Program.desc`` / ``serialize_to_string``
produce the wire-compatible ``ProgramDesc`` protobuf (framework/proto.py).
"""
from __future__ import annotations

import contextlib
import copy
import re
from collections import OrderedDict

import numpy as np

from ..framework import core
from ..framework import registry as R
from ..framework.proto import AttrType, BlockDescPB, OpDescPB, ProgramDescPB, VarTypeEnum
from . import unique_name

VarType = VarTypeEnum
GRAD_VAR_SUFFIX = R.GRAD_SUFFIX
TEMP_VAR_NAME = R.TEMP_VAR
EMPTY_VAR_NAME = R.EMPTY_VAR
ZERO_VAR_SUFFIX = "@ZERO"
CONTROL_DEP_VAR_PREFIX = "@CTRL_DEP@"


def grad_var_name(var_name):
    return var_name + GRAD_VAR_SUFFIX


def convert_np_dtype_to_dtype_(np_dtype):
    return core.convert_dtype(np_dtype)


def dtype_is_floating(dtype):
    return core.convert_dtype(dtype) in (VarType.FP16, VarType.FP32, VarType.FP64, VarType.BF16)


_name_scope_stack = []


@contextlib.contextmanager
def name_scope(prefix=None):
    _name_scope_stack.append(prefix or "")
    try:
        yield
    finally:
        _name_scope_stack.pop()


def _current_name_scope():
    return "/".join(p for p in _name_scope_stack if p)


# =================================================================== Variable


class Variable:
    """A symbolic variable of a Block (framework.py:207)."""

    def __init__(self, block, type=VarType.LOD_TENSOR, name=None, shape=None, dtype=None, lod_level=None,
                 capacity=None, persistable=None, error_clip=None, stop_gradient=False, is_data=False,
                 **kwargs):
        self.block = block
        self.error_clip = error_clip
        if name is None:
            name = unique_name.generate("_generated_var")
        existing = block.vars.get(name)
        self.name = name
        self.type = type
        self.shape = tuple(shape) if shape is not None else (existing.shape if existing else ())
        self.dtype = core.convert_dtype(dtype) if dtype is not None else (
            existing.dtype if existing else VarType.FP32)
        self.lod_level = lod_level if lod_level is not None else (existing.lod_level if existing else 0)
        self.persistable = bool(persistable) if persistable is not None else (
            existing.persistable if existing else False)
        self.capacity = capacity
        self.stop_gradient = stop_gradient
        self.is_data = is_data
        self.op = None
        block.vars[name] = self

    # API parity helpers
    @property
    def desc(self):
        return _VarDescView(self)

    def to_string(self, throw_on_error=False, with_details=False):
        s = f"var {self.name} : {_type_name(self.type)}.shape{list(self.shape)}.dtype({core.dtype_to_str(self.dtype)})" \
            f".lod_level({self.lod_level})"
        if with_details:
            s += f" persistable={self.persistable} stop_gradient={self.stop_gradient}"
        return s

    __str__ = to_string

    def __repr__(self):
        return self.to_string()

    def set_desc(self, input):
        pass

    def _set_error_clip(self, error_clip):
        self.error_clip = error_clip

    def to_proto(self):
        from ..framework.proto import VarDescPB

        d = VarDescPB(name=self.name, persistable=self.persistable)
        d.type.type = self.type
        if self.type in (VarType.LOD_TENSOR,):
            d.type.lod_tensor.tensor.data_type = self.dtype
            d.type.lod_tensor.tensor.dims.extend([int(s) for s in self.shape])
            d.type.lod_tensor.lod_level = int(self.lod_level or 0)
        elif self.type == VarType.SELECTED_ROWS:
            d.type.selected_rows.data_type = self.dtype
            d.type.selected_rows.dims.extend([int(s) for s in self.shape])
        elif self.type == VarType.LOD_TENSOR_ARRAY:
            d.type.tensor_array.tensor.data_type = self.dtype
            d.type.tensor_array.tensor.dims.extend([int(s) for s in self.shape])
            d.type.tensor_array.lod_level = int(self.lod_level or 0)
        return d


class _VarDescView:
    def __init__(self, v):
        self._v = v

    def name(self):
        return self._v.name

    def shape(self):
        return list(self._v.shape)

    def set_shape(self, s):
        self._v.shape = tuple(s)

    def dtype(self):
        return self._v.dtype

    def set_dtype(self, d):
        self._v.dtype = core.convert_dtype(d)

    def type(self):
        return self._v.type

    def set_type(self, t):
        self._v.type = t

    def lod_level(self):
        return self._v.lod_level

    def set_lod_level(self, l):
        self._v.lod_level = l

    def persistable(self):
        return self._v.persistable

    def set_persistable(self, p):
        self._v.persistable = p

    def serialize_to_string(self):
        return self._v.to_proto().SerializeToString()


def _type_name(t):
    for k, v in vars(VarType).items():
        if v == t and not k.startswith("_"):
            return k
    return str(t)


class Parameter(Variable):
    """Persistable trainable variable (framework.py:1942)."""

    def __init__(self, block, shape, dtype, **kwargs):
        if shape is None or dtype is None:
            raise ValueError("Parameter must have shape and dtype")
        for s in shape:
            if s < 0:
                raise ValueError("Parameter shape must be fully known")
        Variable.__init__(self, block, persistable=True, shape=shape, dtype=dtype, **kwargs)
        self.trainable = kwargs.get("trainable", True)
        self.optimize_attr = kwargs.get("optimize_attr", {"learning_rate": 1.0})
        self.regularizer = kwargs.get("regularizer", None)
        self.gradient_clip_attr = kwargs.get("gradient_clip_attr", None)
        self.do_model_average = kwargs.get("do_model_average", None)

    def to_string(self, throw_on_error=False, with_details=False):
        s = Variable.to_string(self, throw_on_error, with_details)
        if with_details:
            s += f" trainable={self.trainable}"
        return s

    __str__ = to_string

    def astype(self, dtype):
        from .layers import tensor as T

        return T.cast(self, dtype)


# =================================================================== Operator


def _as_list(x):
    if x is None:
        return []
    if isinstance(x, (list, tuple)):
        return list(x)
    return [x]


def _var_name(v):
    if isinstance(v, Variable):
        return v.name
    if isinstance(v, str):
        return v
    raise TypeError(f"expected Variable or name, got {type(v)}")


class Operator:
    """One op of a Block (framework.py:496)."""

    OP_WITHOUT_KERNEL_SET = {"feed", "fetch", "save", "load", "recurrent", "go", "rnn_memory_helper_grad",
                             "conditional_block", "while", "send", "recv", "listen_and_serv", "parallel_do",
                             "save_combine", "load_combine", "ncclInit", "channel_create", "channel_close",
                             "channel_send", "channel_recv", "select", "checkpoint_notify", "gen_nccl_id"}

    def __init__(self, block, desc=None, type=None, inputs=None, outputs=None, attrs=None):
        self.block = block
        if type is None:
            raise ValueError("Operator type must be set")
        self.type = type
        info = R.get_op_info(type)
        self._info = info
        self.inputs = OrderedDict()
        self.outputs = OrderedDict()
        for slot, args in (inputs or {}).items():
            self.inputs[slot] = [_var_name(a) for a in _as_list(args)]
        for slot, args in (outputs or {}).items():
            self.outputs[slot] = [_var_name(a) for a in _as_list(args)]
        for s in info.inputs:
            if s.name not in self.inputs and not s.dispensable:
                self.inputs[s.name] = []
            if len(self.inputs.get(s.name, [])) > 1 and not s.duplicable:
                raise ValueError(f"op {type}: input {s.name} is not duplicable")
        self.attrs = OrderedDict()
        for k, d in info.attrs.items():
            self.attrs[k] = copy.deepcopy(d)
        for k, v in (attrs or {}).items():
            if v is None:
                continue
            if isinstance(v, Block):
                self.attrs[k] = v
            elif isinstance(v, np.ndarray):
                self.attrs[k] = v.tolist()
            elif isinstance(v, (np.integer,)):
                self.attrs[k] = int(v)
            elif isinstance(v, (np.floating,)):
                self.attrs[k] = float(v)
            else:
                self.attrs[k] = v
        prog = block.program
        self.attrs.setdefault(R.OP_ROLE_ATTR, prog._current_role)
        if prog._op_role_var and R.OP_ROLE_VAR_ATTR not in self.attrs:
            self.attrs[R.OP_ROLE_VAR_ATTR] = list(prog._op_role_var)
        for slot, names in self.outputs.items():
            for n in names:
                v = block._find_var_recursive(n)
                if v is not None and v.op is None:
                    v.op = self
        if type not in ("feed", "fetch"):
            self._infer_shape()

    # ---- compile-time inference
    def _infer_shape(self):
        info = self._info
        if info.no_infer or info.kernel is None:
            return
        in_descs = {}
        for slot, names in self.inputs.items():
            lst = []
            for n in names:
                v = self.block._find_var_recursive(n)
                if v is None or v.type not in (VarType.LOD_TENSOR, VarType.SELECTED_ROWS) or v.shape is None:
                    lst.append(None)
                else:
                    lst.append((list(v.shape), v.dtype, v.lod_level))
            in_descs[slot] = lst
        # all required inputs must be known
        for s in info.inputs:
            vals = in_descs.get(s.name, [])
            if not s.dispensable and (not vals or any(d is None for d in vals)):
                return
            if any(d is not None and len(d[0]) == 0 and False for d in vals):
                return
        try:
            if info.infer_shape is not None:
                res = info.infer_shape(in_descs, self.attrs)
            else:
                res = R.infer_shapes_meta(info, in_descs, {k: list(v) for k, v in self.outputs.items()},
                                          self._plain_attrs())
        except Exception:
            res = self._lod_fallback_shapes(info, in_descs)
            if not res:
                return
        has_lod_in = any(d is not None and d[2] for lst in in_descs.values() for d in lst)
        if has_lod_in and not info.share_lod and res:
            # a LoD-changing op (sequence_pool/expand, ...): its row count depends on
            # the LoD, which compile time does not know
            res = {slot: [((-1,) + tuple(d[0][1:]), d[1]) if (d is not None and len(d[0])) else d for d in lst]
                   for slot, lst in res.items()}
        for slot, lst in (res or {}).items():
            for n, d in zip(self.outputs.get(slot, []), lst):
                if d is None or n == EMPTY_VAR_NAME:
                    continue
                v = self.block._find_var_recursive(n)
                if v is None:
                    continue
                shape, vt = d
                v.shape = tuple(shape)
                v.dtype = vt
                if v.lod_level == 0:
                    src = next((self.block._find_var_recursive(x) for x in self.input_arg_names), None)
                    if src is not None and src.lod_level and shape and src.shape and \
                            (shape[0] == src.shape[0]) and info.share_lod:
                        v.lod_level = src.lod_level

    def _lod_fallback_shapes(self, info, in_descs):
        """Meta execution failed (data-dependent LoD op): Out = [-1] + X.shape[1:]."""
        x = (in_descs.get("X") or [None])[0]
        if x is None or "Out" not in self.outputs:
            return None
        return {"Out": [((-1,) + tuple(x[0][1:]), x[1])]}

    def _plain_attrs(self):
        return {k: (v.idx if isinstance(v, Block) else v) for k, v in self.attrs.items()}

    # ---- accessors (API.spec)
    def input(self, name):
        return list(self.inputs.get(name, []))

    def output(self, name):
        return list(self.outputs.get(name, []))

    @property
    def input_names(self):
        return list(self.inputs.keys())

    @property
    def output_names(self):
        return list(self.outputs.keys())

    @property
    def input_arg_names(self):
        return [n for v in self.inputs.values() for n in v]

    @property
    def output_arg_names(self):
        return [n for v in self.outputs.values() for n in v]

    def rename_input(self, old_name, new_name):
        for k, v in self.inputs.items():
            self.inputs[k] = [new_name if n == old_name else n for n in v]

    def rename_output(self, old_name, new_name):
        for k, v in self.outputs.items():
            self.outputs[k] = [new_name if n == old_name else n for n in v]

    def has_attr(self, name):
        return name in self.attrs

    def attr(self, name):
        return self.attrs.get(name)

    def attr_type(self, name):
        return R.attr_type_of(self.attrs[name]) if not isinstance(self.attrs[name], Block) else AttrType.BLOCK

    def set_attr(self, name, val):
        self.attrs[name] = val

    _set_attr = set_attr

    @property
    def attr_names(self):
        return list(self.attrs.keys())

    def all_attrs(self):
        return OrderedDict((k, v) for k, v in self.attrs.items())

    def block_attr(self, name):
        return self.attrs[name]

    def block_attr_id(self, name):
        return self.attrs[name].idx

    def blocks_attr(self, name):
        return list(self.attrs[name])

    def blocks_attr_ids(self, name):
        return [b.idx for b in self.attrs[name]]

    def has_kernel(self, op_type):
        return op_type not in self.OP_WITHOUT_KERNEL_SET

    @property
    def desc(self):
        return self

    def to_proto(self):
        d = OpDescPB(type=self.type)
        for k, v in self.inputs.items():
            d.inputs.add(parameter=k, arguments=list(v))
        for k, v in self.outputs.items():
            d.outputs.add(parameter=k, arguments=list(v))
        for k, v in self.attrs.items():
            a = d.attrs.add(name=k, type=AttrType.INT)
            _set_pb_attr(a, v)
        return d

    def to_string(self, throw_on_error=False):
        ins = ", ".join(f"{k}={v}" for k, v in self.inputs.items())
        outs = ", ".join(f"{k}={v}" for k, v in self.outputs.items())
        attrs = ", ".join(f"{k}={v if not isinstance(v, Block) else 'block[%d]' % v.idx}"
                          for k, v in self.attrs.items() if k not in (R.OP_ROLE_ATTR, R.OP_ROLE_VAR_ATTR))
        return f"{{{outs}}} = {self.type}(inputs={{{ins}}}, {attrs})"

    __str__ = to_string
    __repr__ = to_string


def _set_pb_attr(a, v):
    if isinstance(v, Block):
        a.type = AttrType.BLOCK
        a.block_idx = v.idx
        return
    if isinstance(v, (list, tuple)) and v and all(isinstance(x, Block) for x in v):
        a.type = AttrType.BLOCKS
        a.blocks_idx.extend([b.idx for b in v])
        return
    t = R.attr_type_of(v)
    a.type = t
    if t == AttrType.BOOLEAN:
        a.b = bool(v)
    elif t == AttrType.INT:
        a.i = int(v)
    elif t == AttrType.LONG:
        a.l = int(v)
    elif t == AttrType.FLOAT:
        a.f = float(v)
    elif t == AttrType.STRING:
        a.s = str(v)
    elif t == AttrType.INTS:
        a.ints.extend([int(x) for x in v])
    elif t == AttrType.FLOATS:
        a.floats.extend([float(x) for x in v])
    elif t == AttrType.STRINGS:
        a.strings.extend([str(x) for x in v])
    elif t == AttrType.BOOLEANS:
        a.bools.extend([bool(x) for x in v])


def _get_pb_attr(a, blocks):
    t = a.type
    if t == AttrType.INT:
        return a.i
    if t == AttrType.FLOAT:
        return a.f
    if t == AttrType.STRING:
        return a.s
    if t == AttrType.INTS:
        return list(a.ints)
    if t == AttrType.FLOATS:
        return list(a.floats)
    if t == AttrType.STRINGS:
        return list(a.strings)
    if t == AttrType.BOOLEAN:
        return a.b
    if t == AttrType.BOOLEANS:
        return list(a.bools)
    if t == AttrType.LONG:
        return a.l
    if t == AttrType.BLOCK:
        return ("__block__", a.block_idx)
    if t == AttrType.BLOCKS:
        return ("__blocks__", list(a.blocks_idx))
    return None


# =================================================================== Block


class Block:
    """framework.py:923."""

    def __init__(self, program, idx):
        self.program = program
        self.idx = idx
        self.vars = OrderedDict()
        self.ops = []
        self.parent_idx = -1
        self.forward_block_idx = -1
        self.removed_vars = OrderedDict()

    @property
    def desc(self):
        return self

    def to_string(self, throw_on_error=False, with_details=False):
        lines = [f"block {{ idx: {self.idx} parent_idx: {self.parent_idx}"]
        for v in self.vars.values():
            lines.append("  " + v.to_string(throw_on_error, with_details))
        for op in self.ops:
            lines.append("  " + op.to_string(throw_on_error))
        lines.append("}")
        return "\n".join(lines)

    __str__ = to_string

    @property
    def parent_block(self):
        return self.program.block(self.parent_idx) if self.parent_idx >= 0 else None

    def set_forward_block_idx(self, idx):
        self.forward_block_idx = idx

    def var(self, name):
        if not isinstance(name, str):
            raise TypeError("var name must be str")
        v = self.vars.get(name)
        if v is None:
            raise ValueError(f"var {name} not in this block")
        return v

    def _find_var_recursive(self, name):
        b = self
        while b is not None:
            v = b.vars.get(name)
            if v is not None:
                return v
            b = b.parent_block
        return None

    _var_recursive = _find_var_recursive

    def var_recursive(self, name):
        v = self._find_var_recursive(name)
        if v is None:
            raise ValueError(f"var {name} not found")
        return v

    def has_var(self, name):
        return name in self.vars

    def all_parameters(self):
        return [v for v in self.vars.values() if isinstance(v, Parameter)]

    def iter_parameters(self):
        return (v for v in self.vars.values() if isinstance(v, Parameter))

    def create_var(self, *args, **kwargs):
        v = Variable(self, *args, **kwargs)
        if "initializer" in kwargs and kwargs["initializer"] is not None:
            kwargs["initializer"](v, self)
        return v

    def create_parameter(self, *args, **kwargs):
        global_block = self.program.global_block()
        init = kwargs.pop("initializer", None)
        p = Parameter(global_block, *args, **kwargs)
        if init is not None:
            init(p, self)
        return p

    def rename_var(self, name, new_name):
        v = self.vars.pop(name)
        v.name = new_name
        self.vars[new_name] = v
        for op in self.ops:
            op.rename_input(name, new_name)
            op.rename_output(name, new_name)
        return v

    def remove_var(self, name):
        self.vars.pop(name, None)

    def append_op(self, *args, **kwargs):
        op = Operator(self, None, *args, **kwargs)
        self.ops.append(op)
        return op

    def insert_op(self, index, *args, **kwargs):
        op = Operator(self, None, *args, **kwargs)
        self.ops.insert(index, op)
        return op

    def prepend_op(self, *args, **kwargs):
        op = Operator(self, None, *args, **kwargs)
        self.ops.insert(0, op)
        return op

    def remove_op(self, index):
        self.ops.pop(index)

    def slice_ops(self, start, end):
        return self.ops[start:end]

    def sync_with_cpp(self):
        pass

    def copy_param_info_from(self, other):
        for p in other.iter_parameters():
            v = self.vars.get(p.name)
            if v is None:
                continue
            np_ = Parameter(self, p.shape, p.dtype, type=p.type, lod_level=p.lod_level,
                            stop_gradient=p.stop_gradient, trainable=p.trainable,
                            optimize_attr=p.optimize_attr, regularizer=p.regularizer,
                            gradient_clip_attr=p.gradient_clip_attr, error_clip=p.error_clip, name=p.name)
            self.vars[p.name] = np_

    def to_proto(self):
        d = BlockDescPB(idx=self.idx, parent_idx=self.parent_idx, forward_block_idx=self.forward_block_idx)
        for v in self.vars.values():
            d.vars.append(v.to_proto())
        for op in self.ops:
            d.ops.append(op.to_proto())
        return d


# =================================================================== Program


class Program:
    """framework.py:1407."""

    def __init__(self):
        self.blocks = [Block(self, 0)]
        self.current_block_idx = 0
        self.random_seed = 0
        self._current_role = R.OpRole.Forward
        self._op_role_var = []
        self._version = 0
        self._seed_gen = None

    # role helpers used by optimizer / backward
    @property
    def op_role(self):
        return self._current_role

    @op_role.setter
    def op_role(self, role):
        self._current_role = role

    @property
    def op_role_var(self):
        return self._op_role_var

    @contextlib.contextmanager
    def optimized_guard(self, param_and_grads):
        old_role, old_var = self._current_role, self._op_role_var
        self._current_role = R.OpRole.Optimize
        self._op_role_var = [v.name if isinstance(v, Variable) else v for v in param_and_grads if v is not None]
        try:
            yield
        finally:
            self._current_role, self._op_role_var = old_role, old_var

    _optimized_guard = optimized_guard

    @contextlib.contextmanager
    def _lr_schedule_guard(self):
        old = self._current_role
        self._current_role = R.OpRole.LRSched
        try:
            yield
        finally:
            self._current_role = old

    @contextlib.contextmanager
    def _backward_role_guard(self):
        old = self._current_role
        self._current_role = R.OpRole.Backward
        try:
            yield
        finally:
            self._current_role = old

    def __str__(self):
        return self.to_string(True)

    def to_string(self, throw_on_error=False, with_details=False):
        return "\n".join(b.to_string(throw_on_error, with_details) for b in self.blocks)

    def get_desc(self):
        return _ProgramDescView(self)

    @property
    def desc(self):
        return _ProgramDescView(self)

    def global_block(self):
        return self.blocks[0]

    def block(self, index):
        return self.blocks[index]

    def current_block(self):
        return self.blocks[self.current_block_idx]

    def create_block(self, parent_idx=None):
        new_idx = len(self.blocks)
        parent = self.current_block() if parent_idx is None else self.block(parent_idx)
        b = Block(self, new_idx)
        b.parent_idx = parent.idx
        self.blocks.append(b)
        self.current_block_idx = new_idx
        return b

    def rollback(self):
        self.current_block_idx = self.current_block().parent_idx

    @property
    def num_blocks(self):
        return len(self.blocks)

    def list_vars(self):
        for b in self.blocks:
            yield from b.vars.values()

    def all_parameters(self):
        return self.global_block().all_parameters()

    def clone(self, for_test=False):
        p = Program()
        p.random_seed = self.random_seed
        p.blocks = []
        memo = {}
        for b in self.blocks:
            nb = Block(p, b.idx)
            nb.parent_idx, nb.forward_block_idx = b.parent_idx, b.forward_block_idx
            p.blocks.append(nb)
        for b, nb in zip(self.blocks, p.blocks):
            for name, v in b.vars.items():
                nv = copy.copy(v)
                nv.block = nb
                nv.op = None
                nb.vars[name] = nv
            for op in b.ops:
                nop = copy.copy(op)
                nop.block = nb
                nop.inputs = OrderedDict((k, list(v)) for k, v in op.inputs.items())
                nop.outputs = OrderedDict((k, list(v)) for k, v in op.outputs.items())
                nop.attrs = OrderedDict()
                for k, v in op.attrs.items():
                    if isinstance(v, Block):
                        nop.attrs[k] = p.blocks[v.idx]
                    elif isinstance(v, (list, tuple)) and v and all(isinstance(x, Block) for x in v):
                        nop.attrs[k] = [p.blocks[x.idx] for x in v]
                    else:
                        nop.attrs[k] = copy.deepcopy(v, memo)
                if for_test and "is_test" in nop.attrs:
                    nop.attrs["is_test"] = True
                if for_test and nop.type in ("dropout", "batch_norm") and "is_test" not in nop.attrs:
                    nop.attrs["is_test"] = True
                nb.ops.append(nop)
        if for_test:
            p = p._inference_optimize(prune_read_op=False)
        return p

    def _prune(self, targets):
        return self.prune(targets)

    def prune(self, targets):
        """Keep only ops needed to compute ``targets`` (prune.cc semantics)."""
        if not isinstance(targets, (list, tuple)):
            targets = [targets]
        names = set()
        target_ops = []
        for t in targets:
            if isinstance(t, Variable):
                names.add(t.name)
            elif isinstance(t, Operator):
                target_ops.append(t)
                names.update(t.output_arg_names)
            else:
                names.add(str(t))
        res = self.clone()
        gb = res.global_block()
        keep = []
        needed = set(names)
        for op in reversed(gb.ops):
            if any(n in needed for n in op.output_arg_names) or any(op is t for t in target_ops):
                keep.append(op)
                needed.update(op.input_arg_names)
                for v in op.attrs.values():
                    if isinstance(v, Block):
                        for sop in v.ops:
                            needed.update(sop.input_arg_names)
        gb.ops = list(reversed(keep))
        used = set()
        for b in res.blocks:
            for op in b.ops:
                used.update(op.input_arg_names)
                used.update(op.output_arg_names)
        for n in list(gb.vars.keys()):
            if n not in used and n not in names:
                del gb.vars[n]
        return res

    def _inference_optimize(self, prune_read_op=True):
        res = self
        gb = res.global_block()
        if prune_read_op:
            gb.ops = [op for op in gb.ops if op.type not in ("read", "create_py_reader", "create_double_buffer_reader")]
        for b in res.blocks:
            for op in b.ops:
                if "is_test" in op.attrs:
                    op.attrs["is_test"] = True
        return res

    def inference_optimize(self, export_for_deployment=True):
        return self.clone(for_test=True)

    def copy_data_info_from(self, other):
        for name, v in other.global_block().vars.items():
            if name in self.global_block().vars and v.is_data:
                self.global_block().vars[name].is_data = True

    def copy_param_info_from(self, other):
        self.global_block().copy_param_info_from(other.global_block())

    def _copy_dist_param_info_from(self, other):
        pass

    # ---- serialization
    def to_proto(self):
        d = ProgramDescPB()
        for b in self.blocks:
            d.blocks.append(b.to_proto())
        return d

    def serialize_to_string(self):
        return self.to_proto().SerializeToString()

    @staticmethod
    def parse_from_string(binary_str):
        d = ProgramDescPB.FromString(binary_str)
        return Program.from_proto(d)

    @staticmethod
    def from_proto(d):
        p = Program()
        p.blocks = []
        for bd in d.blocks:
            b = Block(p, bd.idx)
            b.parent_idx = bd.parent_idx
            b.forward_block_idx = bd.forward_block_idx
            p.blocks.append(b)
        for bd, b in zip(d.blocks, p.blocks):
            for vd in bd.vars:
                t = vd.type.type
                shape, dtype, lod = (), VarType.FP32, 0
                if vd.type.HasField("lod_tensor"):
                    shape = tuple(vd.type.lod_tensor.tensor.dims)
                    dtype = vd.type.lod_tensor.tensor.data_type
                    lod = vd.type.lod_tensor.lod_level
                elif vd.type.HasField("selected_rows"):
                    shape = tuple(vd.type.selected_rows.dims)
                    dtype = vd.type.selected_rows.data_type
                elif vd.type.HasField("tensor_array"):
                    shape = tuple(vd.type.tensor_array.tensor.dims)
                    dtype = vd.type.tensor_array.tensor.data_type
                    lod = vd.type.tensor_array.lod_level
                Variable(b, type=t, name=vd.name, shape=shape, dtype=dtype, lod_level=lod,
                         persistable=vd.persistable)
            for od in bd.ops:
                op = Operator.__new__(Operator)
                op.block = b
                op.type = od.type
                try:
                    op._info = R.get_op_info(od.type)
                except KeyError:
                    op._info = None
                op.inputs = OrderedDict((v.parameter, list(v.arguments)) for v in od.inputs)
                op.outputs = OrderedDict((v.parameter, list(v.arguments)) for v in od.outputs)
                op.attrs = OrderedDict()
                for a in od.attrs:
                    val = _get_pb_attr(a, p.blocks)
                    if isinstance(val, tuple) and val and val[0] == "__block__":
                        val = p.blocks[val[1]]
                    elif isinstance(val, tuple) and val and val[0] == "__blocks__":
                        val = [p.blocks[i] for i in val[1]]
                    op.attrs[a.name] = val
                b.ops.append(op)
        return p

    # ---- seeds
    @property
    def random_seed(self):
        return self._seed

    @random_seed.setter
    def random_seed(self, s):
        self._seed = int(s)


class _ProgramDescView:
    """Subset of the C++ ProgramDesc binding used by user code."""

    def __init__(self, p):
        self._p = p

    def serialize_to_string(self):
        return self._p.serialize_to_string()

    def num_blocks(self):
        return len(self._p.blocks)

    def block(self, i):
        return self._p.blocks[i]

    def append_block(self, parent):
        return self._p.create_block(parent.idx if hasattr(parent, "idx") else parent)


# =================================================================== defaults

_main_program_ = Program()
_startup_program_ = Program()


def default_startup_program():
    return _startup_program_


def default_main_program():
    return _main_program_


def switch_main_program(program):
    global _main_program_
    prev = _main_program_
    _main_program_ = program
    return prev


def switch_startup_program(program):
    global _startup_program_
    prev = _startup_program_
    _startup_program_ = program
    return prev


@contextlib.contextmanager
def program_guard(main_program, startup_program=None):
    if not isinstance(main_program, Program):
        raise TypeError("main_program should be Program")
    main_program = switch_main_program(main_program)
    if startup_program is not None:
        startup_program = switch_startup_program(startup_program)
    try:
        yield
    finally:
        switch_main_program(main_program)
        if startup_program is not None:
            switch_startup_program(startup_program)


def get_var(name, program=None):
    if program is None:
        program = default_main_program()
    return program.global_block().var(name)
