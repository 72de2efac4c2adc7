"""Control-flow layers (python/paddle/fluid/layers/control_flow.py: While :655,
IfElse :1412, Switch, StaticRNN :430, array ops, LoD rank-table ops, Print).

Sub-blocks are real Blocks of the Program; the ``while`` / ``conditional_block``
kernels re-enter the interpreter on them (framework/executor.py).
"""
from __future__ import annotations

import contextlib

from ...framework import core
from ..framework import Variable, default_main_program
from ..layer_helper import LayerHelper
from .layer_utils import simple_op
from .tensor import fill_constant

__all__ = ["While", "Switch", "increment", "array_write", "create_array", "less_than", "less_equal",
           "greater_than", "greater_equal", "equal", "not_equal", "array_read", "array_length", "IfElse",
           "ConditionalBlock", "StaticRNN", "Print", "is_empty", "lod_rank_table", "max_sequence_len",
           "lod_tensor_to_array", "array_to_lod_tensor", "shrink_memory", "reorder_lod_tensor_by_rank",
           "split_lod_tensor", "merge_lod_tensor"]


def increment(x, value=1.0, in_place=True):
    helper = LayerHelper("increment", **locals())
    out = x if in_place else helper.create_variable_for_type_inference(dtype=x.dtype)
    helper.append_op(type="increment", inputs={"X": [x]}, outputs={"Out": [out]}, attrs={"step": float(value)})
    return out


def _cmp(op, x, y, cond=None):
    helper = LayerHelper(op)
    if cond is None:
        cond = helper.create_variable_for_type_inference(dtype="bool")
        cond.stop_gradient = True
    helper.append_op(type=op, inputs={"X": [x], "Y": [y]}, outputs={"Out": [cond]})
    return cond


def less_than(x, y, force_cpu=None, cond=None):
    return _cmp("less_than", x, y, cond)


def less_equal(x, y, cond=None):
    return _cmp("less_equal", x, y, cond)


def greater_than(x, y, cond=None):
    return _cmp("greater_than", x, y, cond)


def greater_equal(x, y, cond=None):
    return _cmp("greater_equal", x, y, cond)


def equal(x, y, cond=None):
    return _cmp("equal", x, y, cond)


def not_equal(x, y, cond=None):
    return _cmp("not_equal", x, y, cond)


def create_array(dtype):
    helper = LayerHelper("array", **locals())
    return helper.create_variable(name=f"{helper.name}.out", type=core.VT.LOD_TENSOR_ARRAY, dtype=dtype)


def array_write(x, i, array=None):
    helper = LayerHelper("array_write", **locals())
    if array is None:
        array = helper.create_variable(name=f"{helper.name}.out", type=core.VT.LOD_TENSOR_ARRAY, dtype=x.dtype)
    helper.append_op(type="write_to_array", inputs={"X": [x], "I": [i]}, outputs={"Out": [array]})
    return array


def array_read(array, i):
    helper = LayerHelper("array_read", **locals())
    out = helper.create_variable_for_type_inference(dtype=array.dtype)
    helper.append_op(type="read_from_array", inputs={"X": [array], "I": [i]}, outputs={"Out": [out]})
    return out


def array_length(array):
    return simple_op("lod_array_length", {"X": [array]}, dtype="int64", stop_gradient=True)


def Print(input, first_n=-1, message=None, summarize=-1, print_tensor_name=True, print_tensor_type=True,
          print_tensor_shape=True, print_tensor_lod=True, print_phase="both"):
    helper = LayerHelper("print", **locals())
    out = helper.create_variable_for_type_inference(dtype=input.dtype)
    helper.append_op(type="print", inputs={"In": input}, outputs={"Out": out},
                     attrs={"first_n": first_n, "summarize": summarize, "message": message or "",
                            "print_phase": print_phase.upper()})
    return out


def is_empty(x, cond=None):
    return simple_op("is_empty", {"X": [x]}, dtype="bool", stop_gradient=True)


def lod_rank_table(x, level=0):
    helper = LayerHelper("lod_rank_table", **locals())
    table = helper.create_variable(type=core.VT.LOD_RANK_TABLE, name=f"{helper.name}.out")
    helper.append_op(type="lod_rank_table", inputs={"X": x}, outputs={"Out": table}, attrs={"level": level})
    return table


def max_sequence_len(rank_table):
    return simple_op("max_sequence_len", {"RankTable": rank_table}, dtype="int64", stop_gradient=True)


def lod_tensor_to_array(x, table):
    helper = LayerHelper("lod_tensor_to_array", **locals())
    array = helper.create_variable(name=f"{helper.name}.out", type=core.VT.LOD_TENSOR_ARRAY, dtype=x.dtype)
    helper.append_op(type="lod_tensor_to_array", inputs={"X": x, "RankTable": table}, outputs={"Out": array})
    return array


def array_to_lod_tensor(x, table):
    return simple_op("array_to_lod_tensor", {"X": x, "RankTable": table}, dtype=x.dtype)


def shrink_memory(x, i, table):
    return simple_op("shrink_rnn_memory", {"X": [x], "I": [i], "RankTable": [table]})


def reorder_lod_tensor_by_rank(x, rank_table):
    return simple_op("reorder_lod_tensor_by_rank", {"X": [x], "RankTable": [rank_table]})


def split_lod_tensor(input, mask, level=0):
    helper = LayerHelper("split_lod_tensor", **locals())
    t = helper.create_variable_for_type_inference(dtype=input.dtype)
    f = helper.create_variable_for_type_inference(dtype=input.dtype)
    helper.append_op(type="split_lod_tensor", inputs={"X": input, "Mask": mask},
                     outputs={"OutTrue": t, "OutFalse": f}, attrs={"level": level})
    return t, f


def merge_lod_tensor(in_true, in_false, x, mask, level=0):
    return simple_op("merge_lod_tensor", {"X": x, "Mask": mask, "InTrue": in_true, "InFalse": in_false},
                     {"level": level}, dtype=in_true.dtype)


class BlockGuard:
    def __init__(self, main_program):
        self.main_program = main_program

    def __enter__(self):
        self.main_program.create_block()

    def __exit__(self, exc_type, exc_val, exc_tb):
        self.main_program.rollback()
        return exc_type is None


def _outer_vars_written(block, parent):
    """Vars written inside ``block`` that live in an enclosing block."""
    inner, outs = set(block.vars.keys()), []
    for op in block.ops:
        for n in op.output_arg_names:
            if n not in inner and parent._find_var_recursive(n) is not None and n not in outs:
                outs.append(n)
    reads = []
    for op in block.ops:
        for n in op.input_arg_names:
            if n not in inner and parent._find_var_recursive(n) is not None and n not in reads:
                reads.append(n)
    return reads, outs


class While:
    """while (cond) { block }  -- ``with While(cond).block(): ...``"""

    def __init__(self, cond, is_test=False, name=None):
        self.helper = LayerHelper("while", name=name)
        self.cond_var = cond
        self.is_test = is_test

    @contextlib.contextmanager
    def block(self):
        prog = self.helper.main_program
        parent = prog.current_block()
        sub = prog.create_block()
        try:
            yield
        finally:
            prog.rollback()
            reads, outs = _outer_vars_written(sub, parent)
            step_scope = parent.create_var(type=core.VT.STEP_SCOPES)
            parent.append_op(type="while", inputs={"X": reads, "Condition": [self.cond_var]},
                             outputs={"Out": outs, "StepScopes": [step_scope]},
                             attrs={"sub_block": sub, "is_test": self.is_test})


class ConditionalBlock:
    def __init__(self, inputs, is_scalar_condition=False, name=None):
        self.inputs = inputs
        self.is_scalar_condition = is_scalar_condition
        self.helper = LayerHelper("conditional_block", name=name)

    @contextlib.contextmanager
    def block(self):
        prog = self.helper.main_program
        parent = prog.current_block()
        sub = prog.create_block()
        try:
            yield
        finally:
            prog.rollback()
            reads, outs = _outer_vars_written(sub, parent)
            scope_var = parent.create_var(type=core.VT.STEP_SCOPES)
            parent.append_op(type="conditional_block", inputs={"X": reads, "Cond": self.inputs},
                             outputs={"Out": outs, "Scope": [scope_var]},
                             attrs={"sub_block": sub, "is_scalar_condition": self.is_scalar_condition})


class Switch:
    """Switch-case on scalar boolean conditions (used by piecewise LR decay)."""

    def __init__(self, name=None):
        self.helper = LayerHelper("switch", name=name)
        self.pre_not_conditions = []
        self.inside_scope = False

    @contextlib.contextmanager
    def case(self, condition):
        from .ops import logical_and, logical_not

        if not self.pre_not_conditions:
            cond = condition
            not_cond = logical_not(x=condition)
        else:
            pre = self.pre_not_conditions[-1]
            not_cond = logical_and(x=pre, y=logical_not(x=condition))
            cond = logical_and(x=pre, y=condition)
        self.pre_not_conditions.append(not_cond)
        cb = ConditionalBlock([cond], is_scalar_condition=True)
        with cb.block():
            yield

    @contextlib.contextmanager
    def default(self):
        cb = ConditionalBlock([self.pre_not_conditions[-1]], is_scalar_condition=True)
        with cb.block():
            yield

    def __enter__(self):
        self.inside_scope = True
        return self

    def __exit__(self, *a):
        self.inside_scope = False
        return False


class IfElse:
    """Row-wise if/else on a boolean mask (split_lod_tensor / merge_lod_tensor)."""

    def __init__(self, cond, name=None):
        self.cond = cond
        self.helper = LayerHelper("ifelse", name=name)
        self.input_table = {}
        self.outputs = {True: [], False: []}
        self._branch = None

    def input(self, x):
        if self._branch is None:
            raise ValueError("IfElse.input must be called inside true_block/false_block")
        if x.name not in self.input_table:
            t, f = split_lod_tensor(x, self.cond)
            self.input_table[x.name] = (t, f)
        return self.input_table[x.name][0 if self._branch else 1]

    @contextlib.contextmanager
    def true_block(self):
        self._branch = True
        yield
        self._branch = None

    @contextlib.contextmanager
    def false_block(self):
        self._branch = False
        yield
        self._branch = None

    def output(self, *outs):
        self.outputs[self._branch].extend(outs)

    def __call__(self):
        res = []
        for t, f in zip(self.outputs[True], self.outputs[False]):
            ref = next(iter(self.input_table.values()))
            res.append(merge_lod_tensor(t, f, ref[0], self.cond))
        return res


class StaticRNN:
    """Fixed-length RNN unrolled over the time-major first dimension.

    Built as an unrolled sub-graph (each step's ops appended to the main block):
    ``step_input`` slices step t, ``memory`` carries state, ``step_output``
    collects per-step outputs which ``__call__`` stacks along dim 0.
    """

    def __init__(self, name=None):
        self.helper = LayerHelper("static_rnn", name=name)
        self._inputs = []
        self._mems = []
        self._outputs = []
        self._step_fn = None
        self._recording = False

    @contextlib.contextmanager
    def step(self):
        self._recording = True
        prog = self.helper.main_program
        blk = prog.current_block()
        start = len(blk.ops)
        yield
        self._recording = False
        self._template = blk.ops[start:]
        del blk.ops[start:]
        self._unroll(blk)

    def step_input(self, x):
        v = self.helper.create_variable_for_type_inference(x.dtype)
        v.shape = tuple(x.shape[1:])
        self._inputs.append((x, v))
        return v

    def memory(self, init=None, shape=None, batch_ref=None, init_value=0.0, init_batch_dim_idx=0,
               ref_batch_dim_idx=1):
        if init is None:
            from .tensor import fill_constant_batch_size_like

            init = fill_constant_batch_size_like(batch_ref, [-1] + list(shape[1:]) if shape else [-1], "float32",
                                                 init_value, ref_batch_dim_idx, init_batch_dim_idx)
        m = self.helper.create_variable_for_type_inference(init.dtype)
        m.shape = init.shape
        self._mems.append([m, init, None])
        return m

    def update_memory(self, mem, var):
        for e in self._mems:
            if e[0] is mem:
                e[2] = var

    def step_output(self, o):
        self._outputs.append(o)

    output = step_output

    def _unroll(self, blk):
        from .nn import slice as slice_l, squeeze, stack

        T = self._inputs[0][0].shape[0]
        cur = {m[0].name: m[1].name for m in self._mems}
        outs = {o.name: [] for o in self._outputs}
        for t in range(T):
            ren = dict(cur)
            for x, v in self._inputs:
                st = squeeze(slice_l(x, axes=[0], starts=[t], ends=[t + 1]), axes=[0])
                ren[v.name] = st.name
            for op in self._template:
                ins = {k: [ren.get(n, n) for n in v] for k, v in op.inputs.items()}
                outs_map = {}
                for k, v in op.outputs.items():
                    new = []
                    for n in v:
                        nn_ = f"{n}@step{t}"
                        src = blk._find_var_recursive(n)
                        blk.create_var(name=nn_, dtype=src.dtype if src else None,
                                       shape=src.shape if src else None)
                        ren[n] = nn_
                        new.append(nn_)
                    outs_map[k] = new
                blk.append_op(type=op.type, inputs=ins, outputs=outs_map, attrs=dict(op.attrs))
            for m in self._mems:
                cur[m[0].name] = ren.get(m[2].name, m[2].name)
            for o in self._outputs:
                outs[o.name].append(blk.var(ren[o.name]))
        self._result = [stack(outs[o.name], axis=0) for o in self._outputs]

    def __call__(self, *args, **kwargs):
        return self._result[0] if len(self._result) == 1 else self._result
