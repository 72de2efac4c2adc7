"""Program-level reverse-mode autodiff (python/paddle/fluid/backward.py).

Same algorithm and naming as the reference:
  * loss@GRAD = 1 via a ``fill_constant`` tagged Backward|Loss (backward.py:567);
  * walk the op path in reverse, asking the registry for grad op descs
    (``core.get_grad_op_desc`` == registry.make_grad_op_descs, backward.py:368);
  * grads produced by several ops are renamed ``x@GRAD@RENAME@k`` and summed with
    a ``sum`` op (``_addup_repetitive_outputs_``, backward.py:135);
  * grad ops whose outputs are all unneeded are dropped (``_remove_no_grad_branch_``);
  * ``@GRAD`` vars are created with the forward var's shape/dtype
    (``_append_backward_vars_``, backward.py:393);
  * ``op_role_var = [param, grad]`` marks the op producing each parameter gradient
    (consumed by the data-parallel graph builder).
"""
from __future__ import annotations

import collections

from ..framework import registry as R
from . import unique_name
from .framework import Parameter, Program, Variable

GRAD = R.GRAD_SUFFIX


def _strip_grad_suffix_(name):
    pos = name.find(GRAD)
    return name[:pos] if pos != -1 else name


def _append_grad_suffix_(name):
    return name + GRAD


class _GradOp:
    """Lightweight op-desc record used while building the backward pass."""

    def __init__(self, type, inputs, outputs, attrs):
        self.type = type
        self.inputs = collections.OrderedDict((k, list(v)) for k, v in inputs.items())
        self.outputs = collections.OrderedDict((k, list(v)) for k, v in outputs.items())
        self.attrs = dict(attrs)

    def input_arg_names(self):
        return [n for v in self.inputs.values() for n in v]

    def output_arg_names(self):
        return [n for v in self.outputs.values() for n in v]

    def rename_output(self, old, new):
        for k, v in self.outputs.items():
            self.outputs[k] = [new if n == old else n for n in v]

    def rename_input(self, old, new):
        for k, v in self.inputs.items():
            self.inputs[k] = [new if n == old else n for n in v]


def _get_stop_gradients_(program):
    no_grad = collections.defaultdict(set)
    for b in program.blocks:
        for v in b.vars.values():
            if v.stop_gradient:
                no_grad[b.idx].add(_append_grad_suffix_(v.name))
    return no_grad


def _find_op_path_(block, outputs, inputs, no_grad_set):
    relevant_ops = [False] * len(block.ops)
    out_names = set(o.name for o in outputs)
    in_names = set(i.name for i in inputs)
    if inputs:
        for i, op in enumerate(block.ops):
            if any(n in in_names for n in op.input_arg_names):
                relevant_ops[i] = True
                in_names.update(op.output_arg_names)
        for i, op in reversed(list(enumerate(block.ops))):
            if relevant_ops[i] and any(n in out_names for n in op.output_arg_names):
                out_names.update(n for n in op.input_arg_names if n not in no_grad_set)
            else:
                relevant_ops[i] = False
        return [op for i, op in enumerate(block.ops) if relevant_ops[i]]
    path = []
    for op in reversed(block.ops):
        if any(n in out_names for n in op.output_arg_names):
            path.append(op)
            out_names.update(n for n in op.input_arg_names if n not in no_grad_set)
    path.reverse()
    return path


def _addup_repetitive_outputs_(op_descs):
    pending_sum_ops = []
    var_rename_count = collections.defaultdict(int)
    renamed_vars = collections.defaultdict(list)
    for idx, op in enumerate(op_descs):
        for var_name in op.input_arg_names():
            if len(renamed_vars[var_name]) > 1:
                pending_sum_ops.append((_GradOp("sum", {"X": renamed_vars[var_name]}, {"Out": [var_name]},
                                                {R.OP_ROLE_ATTR: R.OpRole.Backward}), idx))
                renamed_vars[var_name] = [var_name]
        for var_name in op.output_arg_names():
            if var_name == R.EMPTY_VAR or var_name in op.input_arg_names():
                continue
            if len(renamed_vars[var_name]) == 0:
                renamed_vars[var_name] = [var_name]
            else:
                if len(renamed_vars[var_name]) == 1:
                    new_name = var_name + "@RENAME@" + str(var_rename_count[var_name])
                    var_rename_count[var_name] += 1
                    # rename the first producer and its consumers so far (_rename_arg_)
                    for p in op_descs[:idx]:
                        p.rename_output(var_name, new_name)
                        p.rename_input(var_name, new_name)
                    for p, _ in pending_sum_ops:
                        p.rename_input(var_name, new_name)
                        p.rename_output(var_name, new_name)
                    renamed_vars[var_name][0] = new_name
                new_name = var_name + "@RENAME@" + str(var_rename_count[var_name])
                var_rename_count[var_name] += 1
                op.rename_output(var_name, new_name)
                renamed_vars[var_name].append(new_name)
    for var_name, inputs in renamed_vars.items():
        if len(inputs) > 1:
            pending_sum_ops.append((_GradOp("sum", {"X": inputs}, {"Out": [var_name]},
                                            {R.OP_ROLE_ATTR: R.OpRole.Backward}), len(op_descs)))
    for p in reversed(pending_sum_ops):
        op_descs.insert(p[1], p[0])
    return op_descs


def _remove_no_grad_branch_(op_descs, no_grad_set):
    def can_remove(op):
        outs = [n for n in op.output_arg_names() if n != R.EMPTY_VAR]
        if not outs or all(n in no_grad_set for n in outs):
            return True
        gin = [n for n in op.input_arg_names() if GRAD in n]
        if gin and all(n in no_grad_set for n in gin):
            no_grad_set.update(outs)
            return True
        return False

    res = [op for op in op_descs if not can_remove(op)]
    to_insert = []
    for idx, op in enumerate(res):
        for arg in op.input_arg_names():
            if GRAD in arg and arg in no_grad_set:
                to_insert.append((_GradOp("fill_zeros_like", {"X": [_strip_grad_suffix_(arg)]}, {"Out": [arg]},
                                          {R.OP_ROLE_ATTR: R.OpRole.Backward}), idx))
    for op, idx in reversed(to_insert):
        res.insert(idx, op)
    return res


class _OpView:
    """Adapter so registry grad makers can read a fluid Operator."""

    def __init__(self, op):
        self._op = op
        self.type = op.type

    def input(self, n):
        return self._op.input(n)

    def output(self, n):
        return self._op.output(n)

    def all_attrs(self):
        return {k: v for k, v in self._op.attrs.items()}


_DIFF_TYPES = None


def _differentiable(block, name, no_grad):
    from ..framework import core

    global _DIFF_TYPES
    if _DIFF_TYPES is None:
        _DIFF_TYPES = (core.VT.LOD_TENSOR, core.VT.LOD_TENSOR_ARRAY, core.VT.SELECTED_ROWS)
    if _append_grad_suffix_(name) in no_grad:
        return False
    v = block._find_var_recursive(name)
    if v is None or v.type not in _DIFF_TYPES or v.stop_gradient and v.type != core.VT.LOD_TENSOR_ARRAY:
        return False
    return v.dtype in (core.VT.FP32, core.VT.FP64, core.VT.FP16, core.VT.BF16)


def _while_grad_descs(op, block, no_grad_dict, grad_to_var, callbacks):
    """Reference backward.py:315-392 sub-block recursion + WhileGradOpDescMaker: the
    grad block is a child of the forward sub-block (it reads the step-local
    activations kept in the step scopes) and holds the reversed grad ops of every op
    in the loop body."""
    prog = block.program
    sub = op.attrs["sub_block"]
    saved = prog.current_block_idx
    grad_sub = prog.create_block(parent_idx=sub.idx)
    no_grad_dict[sub.idx] = set(no_grad_dict[sub.idx]) | set(no_grad_dict[block.idx])
    _append_backward_ops_(sub, list(sub.ops), grad_sub, no_grad_dict, grad_to_var, callbacks)
    prog.current_block_idx = saved
    no_grad = no_grad_dict[block.idx]
    xs, outs = list(op.input("X")), list(op.output("Out"))
    x_grads = [_append_grad_suffix_(n) if _differentiable(block, n, no_grad) else R.EMPTY_VAR for n in xs]
    ogs = [_append_grad_suffix_(n) for n in outs if _differentiable(block, n, no_grad)]
    return [dict(type="while_grad",
                 inputs={"X": xs, "Out": outs, "Out@GRAD": ogs, "StepScopes": list(op.output("StepScopes"))},
                 outputs={"X@GRAD": x_grads}, attrs={"sub_block": grad_sub, "original_output_grad": ogs})]


def _cond_block_grad_descs(op, block, no_grad_dict, grad_to_var, callbacks):
    """Reference conditional_block_op.cc ConditionalBlockGradMaker: the grad block is
    a child of the forward sub-block and runs in a child of the scope the forward
    kept (``Scope``) -- only when the forward ran."""
    prog = block.program
    sub = op.attrs["sub_block"]
    saved = prog.current_block_idx
    grad_sub = prog.create_block(parent_idx=sub.idx)
    no_grad_dict[sub.idx] = set(no_grad_dict[sub.idx]) | set(no_grad_dict[block.idx])
    _append_backward_ops_(sub, list(sub.ops), grad_sub, no_grad_dict, grad_to_var, callbacks)
    prog.current_block_idx = saved
    no_grad = no_grad_dict[block.idx]
    xs, outs = list(op.input("X")), list(op.output("Out"))
    x_grads = [_append_grad_suffix_(n) if _differentiable(block, n, no_grad) else R.EMPTY_VAR for n in xs]
    ogs = [_append_grad_suffix_(n) for n in outs if _differentiable(block, n, no_grad)]
    return [dict(type="conditional_block_grad",
                 inputs={"X": xs, "Cond": list(op.input("Cond")), "Out": outs, "Out@GRAD": ogs,
                         "Scope": list(op.output("Scope"))},
                 outputs={"X@GRAD": x_grads},
                 attrs={"sub_block": grad_sub, "is_scalar_condition": op.attrs.get("is_scalar_condition", False)})]


def _recurrent_grad_descs(op, block, no_grad_dict, grad_to_var, callbacks):
    """Reference recurrent_op.cc RecurrentGradOpDescMaker: the grad block is a child
    of the step block (it reads each step's activations from the kept step scopes);
    recurrent_grad links the state gradients step to step and stacks / sums the
    per-step input and parameter gradients (RecurrentGradOp::RunImpl)."""
    prog = block.program
    sub = op.attrs["sub_block"]
    saved = prog.current_block_idx
    grad_sub = prog.create_block(parent_idx=sub.idx)
    no_grad_dict[sub.idx] = set(no_grad_dict[sub.idx]) | set(no_grad_dict[block.idx])
    _append_backward_ops_(sub, list(sub.ops), grad_sub, no_grad_dict, grad_to_var, callbacks)
    prog.current_block_idx = saved
    no_grad = no_grad_dict[block.idx]
    # The gradient of a step output / state arrives from outside the block (row t of
    # the output gradient, the later step's ex-state gradient) as <name>@GRAD@EXT,
    # which recurrent_grad always sets; the block adds it to whatever its own ops
    # accumulated for <name>@GRAD (a state also consumed inside the step), or takes
    # it as is.  Without this the block's sum of its own contributions would
    # overwrite the incoming gradient.
    linked = list(dict.fromkeys(list(op.attrs.get("states", [])) + list(op.output("outputs"))))
    for n in linked:
        gname = _append_grad_suffix_(n)
        ext = gname + "@EXT"
        src = sub._find_var_recursive(n)
        for nm in (ext, gname + "@LOCAL"):
            if not grad_sub.has_var(nm):
                grad_sub.create_var(name=nm, dtype=src.dtype if src is not None else "float32",
                                    shape=src.shape if src is not None else None)
        writers = [i for i, gop in enumerate(grad_sub.ops) if gname in gop.output_arg_names]
        if writers:
            last = writers[-1]
            grad_sub.ops[last].rename_output(gname, gname + "@LOCAL")
            grad_sub.insert_op(last + 1, type="sum", inputs={"X": [gname + "@LOCAL", ext]}, outputs={"Out": [gname]},
                               attrs={R.OP_ROLE_ATTR: R.OpRole.Backward})
        else:
            if not grad_sub.has_var(gname):
                grad_sub.create_var(name=gname, dtype=src.dtype if src is not None else "float32",
                                    shape=src.shape if src is not None else None)
            grad_sub.insert_op(0, type="assign", inputs={"X": [ext]}, outputs={"Out": [gname]},
                               attrs={R.OP_ROLE_ATTR: R.OpRole.Backward})

    def grads(names):
        return [_append_grad_suffix_(n) if _differentiable(block, n, no_grad) else R.EMPTY_VAR for n in names]

    xs, inits, params = list(op.input("inputs")), list(op.input("initial_states")), list(op.input("parameters"))
    outs = list(op.output("outputs"))
    ogs = [_append_grad_suffix_(n) for n in outs if _differentiable(block, n, no_grad)]
    attrs = {k: op.attrs[k] for k in ("ex_states", "states", "reverse", "is_train") if k in op.attrs}
    attrs["sub_block"] = grad_sub
    return [dict(type="recurrent_grad",
                 inputs={"inputs": xs, "initial_states": inits, "parameters": params, "outputs": outs,
                         "outputs@GRAD": ogs, "step_scopes": list(op.output("step_scopes"))},
                 outputs={"inputs@GRAD": grads(xs), "initial_states@GRAD": grads(inits),
                          "parameters@GRAD": grads(params)},
                 attrs=attrs)]


def _split_duplicate_outputs(descs):
    """A grad op that writes the same gradient from two slots (``x * x`` ->
    X@GRAD and Y@GRAD are both x@GRAD) gets the later occurrences renamed and a
    ``sum`` appended, so every grad op produces each name at most once."""
    out = []
    for d in descs:
        seen, extra = {}, []
        outs = {}
        for slot, names in d["outputs"].items():
            new = []
            for n in names:
                if n != R.EMPTY_VAR and n in seen:
                    k = seen[n]
                    seen[n] = k + 1
                    dup = f"{n}@DUP@{k}"
                    extra.append((n, dup))
                    new.append(dup)
                else:
                    seen.setdefault(n, 0)
                    new.append(n)
            outs[slot] = new
        if not extra:
            out.append(d)
            continue
        first = {}
        for n, dup in extra:
            first.setdefault(n, []).append(dup)
        for n, dups in first.items():
            # rename the first occurrence too, then sum all into n
            base = f"{n}@DUP@first"
            for slot, names in outs.items():
                if n in names:
                    names[names.index(n)] = base
                    break
            first[n] = [base] + dups
        out.append(dict(d, outputs=outs))
        for n, parts in first.items():
            out.append(dict(type="sum", inputs={"X": parts}, outputs={"Out": [n]}, attrs={}))
    return out


def _append_backward_ops_(block, ops, target_block, no_grad_dict, grad_to_var, callbacks=None):
    grad_op_descs = []
    no_grad = no_grad_dict[block.idx]
    for op in reversed(ops):
        if op.type == "while":
            descs = _while_grad_descs(op, block, no_grad_dict, grad_to_var, callbacks)
        elif op.type == "conditional_block":
            descs = _cond_block_grad_descs(op, block, no_grad_dict, grad_to_var, callbacks)
        elif op.type == "recurrent":
            descs = _recurrent_grad_descs(op, block, no_grad_dict, grad_to_var, callbacks)
        else:
            descs = R.make_grad_op_descs(_OpView(op), no_grad)
        for d in _split_duplicate_outputs(descs):
            g = _GradOp(d["type"], d["inputs"], d["outputs"], d.get("attrs", {}))
            g.attrs[R.OP_ROLE_ATTR] = R.OpRole.Backward
            g.attrs.pop(R.OP_ROLE_VAR_ATTR, None)
            for n in g.output_arg_names():
                if n != R.EMPTY_VAR:
                    grad_to_var[n] = _strip_grad_suffix_(n)
            grad_op_descs.append(g)
    grad_op_descs = _addup_repetitive_outputs_(grad_op_descs)
    grad_op_descs = _remove_no_grad_branch_(grad_op_descs, no_grad_dict[block.idx])
    new_ops = []
    for g in grad_op_descs:
        # ensure grad vars exist before op construction (shape inference looks them up)
        _create_grad_vars(target_block, g)
        op = target_block.append_op(type=g.type, inputs=dict(g.inputs), outputs=dict(g.outputs), attrs=g.attrs)
        new_ops.append(op)
        if callbacks:
            for cb in callbacks:
                cb(block=target_block, context={})
    return new_ops


def _create_grad_vars(block, g):
    for n in g.output_arg_names() + [x for x in g.input_arg_names() if GRAD in x]:
        if n == R.EMPTY_VAR or block._find_var_recursive(n) is not None:
            continue
        fwd = block._find_var_recursive(_strip_grad_suffix_(n))
        if fwd is not None:
            block.create_var(name=n, shape=fwd.shape, dtype=fwd.dtype, lod_level=fwd.lod_level, type=fwd.type)
        else:
            block.create_var(name=n)


def append_backward(loss, parameter_list=None, no_grad_set=None, callbacks=None):
    """Append backward ops for ``loss``; returns [(param, grad_var)]."""
    assert isinstance(loss, Variable)
    program = loss.block.program
    if no_grad_set is None:
        no_grad_set = set()
    no_grad_set = set(n.name if isinstance(n, Variable) else n for n in no_grad_set)
    no_grad_dict = _get_stop_gradients_(program)
    no_grad_dict[0].update(_append_grad_suffix_(n) for n in no_grad_set)
    root = program.global_block()
    loss_grad = _append_grad_suffix_(loss.name)
    with program._backward_role_guard():
        root.create_var(name=loss_grad, shape=loss.shape, dtype=loss.dtype)
        root.append_op(type="fill_constant", outputs={"Out": [loss_grad]},
                       attrs={"shape": [1], "value": 1.0, "dtype": loss.dtype, "force_cpu": False,
                              R.OP_ROLE_ATTR: R.OpRole.Backward | R.OpRole.Loss})
        block_no_grad = set(_strip_grad_suffix_(n) for n in no_grad_dict[0])
        op_path = _find_op_path_(root, [loss], [], block_no_grad)
        no_grad_dict[0].update(_append_grad_suffix_(n) for n in block_no_grad)
        grad_to_var = {}
        new_ops = _append_backward_ops_(root, op_path, root, no_grad_dict, grad_to_var, callbacks)
    if parameter_list is not None:
        params = [p.name if isinstance(p, Variable) else p for p in parameter_list]
    else:
        params = [p.name for p in program.global_block().all_parameters() if p.trainable]
    params_and_grads = []
    for pname in params:
        gname = _append_grad_suffix_(pname)
        if gname not in grad_to_var and root._find_var_recursive(gname) is None:
            continue
        gvar = root._find_var_recursive(gname)
        if gvar is None:
            continue
        if not any(gname in op.output_arg_names for op in new_ops):
            continue
        p = root.var(pname)
        params_and_grads.append((p, gvar))
        for op in reversed(new_ops):
            if gname in op.output_arg_names:
                op.attrs[R.OP_ROLE_VAR_ATTR] = [pname, gname]
                break
    program._version += 1
    return params_and_grads


def calc_gradient(targets, inputs, target_gradients=None, no_grad_set=None):
    """Gradients of ``targets`` w.r.t. ``inputs`` (backward.py:685)."""
    targets = targets if isinstance(targets, list) else [targets]
    inputs = inputs if isinstance(inputs, list) else [inputs]
    block = targets[0].block
    prog = block.program
    no_grad_set = set(n.name if isinstance(n, Variable) else n for n in (no_grad_set or []))
    no_grad_dict = _get_stop_gradients_(prog)
    no_grad_dict[0].update(_append_grad_suffix_(n) for n in no_grad_set)
    for i in inputs:
        no_grad_dict[0].discard(_append_grad_suffix_(i.name))
    with prog._backward_role_guard():
        if target_gradients is None:
            target_gradients = [None] * len(targets)
        for t, tg in zip(targets, target_gradients):
            gname = _append_grad_suffix_(t.name)
            if tg is None:
                block.create_var(name=gname, shape=t.shape, dtype=t.dtype)
                block.append_op(type="fill_constant_batch_size_like" if t.shape and t.shape[0] == -1
                                else "fill_constant",
                                inputs={"Input": [t]} if t.shape and t.shape[0] == -1 else {},
                                outputs={"Out": [gname]},
                                attrs={"shape": list(t.shape) if t.shape else [1], "value": 1.0, "dtype": t.dtype})
            else:
                block.append_op(type="assign", inputs={"X": [tg]}, outputs={"Out": [gname]})
                if gname not in block.vars:
                    block.create_var(name=gname, shape=t.shape, dtype=t.dtype)
        block_no_grad = set(_strip_grad_suffix_(n) for n in no_grad_dict[0])
        op_path = _find_op_path_(block, targets, inputs, block_no_grad)
        grad_to_var = {}
        _append_backward_ops_(block, op_path, block, no_grad_dict, grad_to_var)
    prog._version += 1
    outs = []
    for i in inputs:
        outs.append(block._find_var_recursive(_append_grad_suffix_(i.name)))
    return outs[0] if len(outs) == 1 else outs


gradients = calc_gradient
