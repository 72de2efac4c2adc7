"""Control-flow layers (python/paddle/fluid/layers/control_flow.py: While :655,
IfElse :1412, Switch, StaticRNN :430, array ops, LoD rank-table ops, Print).

Sub-blocks are real Blocks of the Program; the ``while`` / ``conditional_block``
kernels re-enter the interpreter on them (framework/executor.py).
"""
from __future__ import annotations

import contextlib

from ...framework import core
from .. import unique_name
from ..framework import Variable, default_main_program
from ..layer_helper import LayerHelper
from .layer_utils import simple_op
from .tensor import fill_constant

__all__ = ["While", "Switch", "increment", "array_write", "create_array", "less_than", "less_equal",
           "greater_than", "greater_equal", "equal", "not_equal", "array_read", "array_length", "IfElse",
           "ConditionalBlock", "StaticRNN", "Print", "is_empty", "lod_rank_table", "max_sequence_len",
           "lod_tensor_to_array", "array_to_lod_tensor", "shrink_memory", "reorder_lod_tensor_by_rank",
           "split_lod_tensor", "merge_lod_tensor", "DynamicRNN", "ParallelDo"]


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
    # compile-time WriteToArrayInferShape: the array's desc carries its element shape
    # and LoD level (tensor_array_read_write_op.cc), which array_read hands on
    if not array.shape and x.shape:
        array.shape = tuple(x.shape)
        array.lod_level = x.lod_level
    return array


def array_read(array, i):
    helper = LayerHelper("array_read", **locals())
    out = helper.create_variable_for_type_inference(dtype=array.dtype)
    helper.append_op(type="read_from_array", inputs={"X": [array], "I": [i]}, outputs={"Out": [out]})
    if array.shape:  # ReadFromArrayInferShape (compile time): the element shape of the array
        out.shape = tuple(array.shape)
        out.lod_level = array.lod_level
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


# ---------------------------------------------------------------------------- DynamicRNN
def _parent_op(block, type, inputs, outputs, attrs=None):
    return block.append_op(type=type, inputs=inputs, outputs=outputs, attrs=attrs or {})


class DynamicRNN:
    """RNN over variable-length (LoD) sequences (reference control_flow.py:1542).

    Built from a ``While`` loop over time steps: sequences are sorted by length
    (``lod_rank_table``), split time-major into a tensor array, and at step t only
    the sequences still alive take part (``shrink_rnn_memory``).  Trainable end to
    end: ``fluid.backward`` differentiates the loop through ``while_grad``.

        drnn = DynamicRNN()
        with drnn.block():
            word = drnn.step_input(sentence)
            prev = drnn.memory(shape=[200])
            hidden = fluid.layers.fc(input=[word, prev], size=200, act='relu')
            drnn.update_memory(prev, hidden)
            drnn.output(hidden)
        out = drnn()
    """

    BEFORE_RNN, IN_RNN, AFTER_RNN = 0, 1, 2

    def __init__(self, name=None):
        self.helper = LayerHelper("dynamic_rnn", name=name)
        self.status = DynamicRNN.BEFORE_RNN
        self.lod_rank_table = None
        self.max_seq_len = None
        self.step_idx = None
        # loop indices live on the host (force_cpu, as in the reference): the loop
        # condition and the array slots are read there every step
        self.zero_idx = fill_constant(shape=[1], value=0, dtype="int64", force_cpu=True)
        self.zero_idx.stop_gradient = True
        self.mem_dict = {}
        self.output_array = []
        self.outputs = []
        self.cond = self.helper.create_variable_for_type_inference(dtype="bool")
        self.cond.stop_gradient = False
        self.while_op = While(self.cond)
        self.input_array = []
        self.mem_link = []

    def _parent_block(self):
        prog = self.helper.main_program
        return prog.block(prog.current_block().parent_idx)

    def _assert_in_rnn_block_(self, method):
        if self.status != DynamicRNN.IN_RNN:
            raise ValueError(f"{method} can only be invoked inside rnn block.")

    def _init_zero_idx_(self):
        pass

    def step_input(self, x):
        self._assert_in_rnn_block_("step_input")
        parent = self._parent_block()
        if self.lod_rank_table is None:
            self.lod_rank_table = parent.create_var(name=unique_name.generate("lod_rank_table"),
                                                    type=core.VT.LOD_RANK_TABLE)
            self.lod_rank_table.stop_gradient = True
            _parent_op(parent, "lod_rank_table", {"X": [x]}, {"Out": [self.lod_rank_table]}, {"level": 0})
            self.max_seq_len = parent.create_var(name=unique_name.generate("dynamic_rnn_max_seq_len"),
                                                 dtype="int64", shape=[1])
            self.max_seq_len.stop_gradient = True
            _parent_op(parent, "max_sequence_len", {"RankTable": [self.lod_rank_table]},
                       {"Out": [self.max_seq_len]})
            _parent_op(parent, "less_than", {"X": [self.step_idx], "Y": [self.max_seq_len]},
                       {"Out": [self.cond]})
        input_array = parent.create_var(name=unique_name.generate("dynamic_rnn_input_array"),
                                        type=core.VT.LOD_TENSOR_ARRAY, dtype=x.dtype, shape=x.shape)
        self.input_array.append((input_array, x.dtype))
        _parent_op(parent, "lod_tensor_to_array", {"X": [x], "RankTable": [self.lod_rank_table]},
                   {"Out": [input_array]})
        out = array_read(array=input_array, i=self.step_idx)
        out.shape = x.shape
        return out

    def static_input(self, x):
        self._assert_in_rnn_block_("static_input")
        if self.lod_rank_table is None:
            raise RuntimeError("static_input() must be called after step_input().")
        parent = self._parent_block()
        x_reordered = parent.create_var(name=unique_name.generate("dynamic_rnn_static_input_reordered"),
                                        type=core.VT.LOD_TENSOR, dtype=x.dtype, shape=x.shape)
        _parent_op(parent, "reorder_lod_tensor_by_rank", {"X": [x], "RankTable": [self.lod_rank_table]},
                   {"Out": [x_reordered]})
        out = shrink_memory(x_reordered, self.step_idx, self.lod_rank_table)
        out.shape = x.shape
        return out

    @contextlib.contextmanager
    def block(self):
        if self.status != DynamicRNN.BEFORE_RNN:
            raise ValueError("rnn.block() can only be invoke once")
        self.step_idx = fill_constant(shape=[1], dtype="int64", value=0, force_cpu=True)
        self.step_idx.stop_gradient = False
        self.status = DynamicRNN.IN_RNN
        with self.while_op.block():
            yield
            increment(x=self.step_idx, value=1.0, in_place=True)
            for new_mem, mem_array in self.mem_link:
                array_write(x=new_mem, i=self.step_idx, array=mem_array)
            less_than(x=self.step_idx, y=self.max_seq_len, cond=self.cond)
        self.status = DynamicRNN.AFTER_RNN
        for each in self.output_array:
            o = array_to_lod_tensor(x=each, table=self.lod_rank_table)
            o.shape = each.shape
            self.outputs.append(o)

    def __call__(self, *args, **kwargs):
        if self.status != DynamicRNN.AFTER_RNN:
            raise ValueError("Output of the dynamic RNN can only be visited outside the rnn block.")
        return self.outputs[0] if len(self.outputs) == 1 else self.outputs

    def memory(self, init=None, shape=None, value=0.0, need_reorder=False, dtype="float32"):
        self._assert_in_rnn_block_("memory")
        parent = self._parent_block()
        if init is not None:
            if need_reorder:
                if self.lod_rank_table is None:
                    raise ValueError("If set need_reorder to True, make sure step_input be invoked before memory.")
                init_reordered = parent.create_var(name=unique_name.generate("dynamic_rnn_mem_init_reordered"),
                                                   type=core.VT.LOD_TENSOR, dtype=init.dtype, shape=init.shape)
                _parent_op(parent, "reorder_lod_tensor_by_rank", {"X": [init], "RankTable": [self.lod_rank_table]},
                           {"Out": [init_reordered]})
                init = init_reordered
            mem_array = parent.create_var(name=unique_name.generate("dynamic_rnn_mem_array"),
                                          type=core.VT.LOD_TENSOR_ARRAY, dtype=init.dtype, shape=init.shape)
            _parent_op(parent, "write_to_array", {"X": [init], "I": [self.zero_idx]}, {"Out": [mem_array]})
            retv = array_read(array=mem_array, i=self.step_idx)
            retv.shape = init.shape
            retv = shrink_memory(x=retv, i=self.step_idx, table=self.lod_rank_table)
            retv.shape = init.shape
            self.mem_dict[retv.name] = mem_array
            return retv
        if len(self.input_array) == 0:
            raise ValueError("step_input should be invoked before memory(shape=..., value=...)")
        arr, in_dtype = self.input_array[0]
        in0 = parent.create_var(name=unique_name.generate("in0"), dtype=in_dtype)
        _parent_op(parent, "read_from_array", {"X": [arr], "I": [self.zero_idx]}, {"Out": [in0]})
        init = parent.create_var(name=unique_name.generate("mem_init"), dtype=dtype, shape=[-1] + list(shape))
        init.stop_gradient = True
        _parent_op(parent, "fill_constant_batch_size_like", {"Input": [in0]}, {"Out": [init]},
                   {"shape": [-1] + list(shape), "value": float(value), "dtype": core.convert_dtype(dtype)})
        return self.memory(init=init)

    def update_memory(self, ex_mem, new_mem):
        self._assert_in_rnn_block_("update_memory")
        mem_array = self.mem_dict.get(ex_mem.name)
        if mem_array is None:
            raise ValueError("Please invoke memory before update_memory")
        if self.lod_rank_table is None:
            raise ValueError("Please invoke step_input before update_memory")
        self.mem_link.append((new_mem, mem_array))

    def output(self, *outputs):
        self._assert_in_rnn_block_("output")
        parent = self._parent_block()
        for each in outputs:
            outside_array = parent.create_var(name=unique_name.generate(f"_{self.helper.name}_output_array_"),
                                              type=core.VT.LOD_TENSOR_ARRAY, dtype=each.dtype, shape=each.shape)
            array_write(x=each, i=self.step_idx, array=outside_array)
            self.output_array.append(outside_array)


# ---------------------------------------------------------------------------- ParallelDo
class ParallelDo:
    """Op-level data parallelism over places (reference control_flow.py:230,
    operators/parallel_do_op.cc).  Deprecated in the reference in favour of
    ParallelExecutor; kept for API parity.

    MI355X design: the sub-block is traced once and run on the input as a whole
    on the current place (one process per GPU is the data-parallel unit here; the
    multi-replica split of the reference's threads is what ParallelExecutor /
    ``paddle_amd.distributed`` provide).  ``read_input`` / ``write_output`` keep
    their meaning, so programs written against ParallelDo build and train.
    """

    def __init__(self, places, use_nccl=False, name=None):
        self.helper = LayerHelper("parallel_do", name=name)
        self.places = places
        self.use_nccl = use_nccl
        self.inputs = []
        self.outputs = []

    @contextlib.contextmanager
    def do(self):
        yield

    def parent_block(self):
        prog = self.helper.main_program
        return prog.current_block()

    def read_input(self, var):
        self.inputs.append(var)
        return var

    def write_output(self, var):
        self.outputs.append(var)

    def get_parameters(self):
        return [p for p in self.helper.main_program.global_block().all_parameters()]

    def __call__(self, *args, **kwargs):
        if not self.outputs:
            raise ValueError("ParallelDo: call write_output() inside do()")
        return self.outputs[0] if len(self.outputs) == 1 else self.outputs
