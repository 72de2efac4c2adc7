"""Feed / fetch / save / load operators and control-flow operators.

Parity: paddle/fluid/operators/{feed,fetch,save,load,save_combine,load_combine}_op.cc
(one file per var, or all vars concatenated), controlflow
{while,conditional_block}_op.cc, {lod_rank_table,lod_tensor_to_array,
array_to_lod_tensor,shrink_rnn_memory,split_lod_tensor,merge_lod_tensor,
reorder_lod_tensor_by_rank,max_sequence_len,tensor_array_read_write,
lod_array_length}_op.cc.
"""
from __future__ import annotations

import os

import torch

from ..framework import core
from ..framework import serialization as S
from ..framework.registry import register_op

# ------------------------------------------------------------------ feed / fetch


@register_op("feed", ["X"], ["Out"], {"col": 0}, grad=None, no_infer=True, share_lod=False)
def feed(ctx):
    lst = ctx.input_value("X")
    v = lst[ctx.attr("col")]
    if isinstance(v, core.LoDTensor) and v.tensor is not None and v.tensor.device != ctx.device:
        v = core.LoDTensor(v.tensor.to(ctx.device, non_blocking=True), v.lod())
    ctx.set_output("Out", v)


@register_op("fetch", ["X"], ["Out"], {"col": 0}, grad=None, no_infer=True, share_lod=False)
def fetch(ctx):
    v = ctx.input_value("X")
    name = ctx.op.output("Out")[0] if ctx.op else "fetch"
    var = ctx.scope.find_var(name) if ctx.scope is not None else None
    lst = var.get() if var is not None and var.get() is not None else []
    col = ctx.attr("col")
    while len(lst) <= col:
        lst.append(None)
    lst[col] = v
    if var is not None:
        var.set(lst)


# ------------------------------------------------------------------ save / load


def _ensure_dir(path):
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)


@register_op("save", ["X"], [], {"overwrite": True, "save_as_fp16": False, "file_path": ""}, grad=None,
             no_infer=True)
def save(ctx):
    path = ctx.attr("file_path")
    if os.path.exists(path) and not ctx.attr("overwrite"):
        raise RuntimeError(f"{path} exists; set overwrite=True")
    _ensure_dir(path)
    v = ctx.input_value("X")
    with open(path, "wb") as f:
        if isinstance(v, core.SelectedRows):
            S.write_selected_rows(f, v)
        else:
            if ctx.attr("save_as_fp16") and v.tensor.is_floating_point():
                v = core.LoDTensor(v.tensor.half(), v.lod())
            S.write_lod_tensor(f, v)


@register_op("load", [], ["Out"], {"file_path": "", "load_as_fp16": False}, grad=None, no_infer=True)
def load(ctx):
    with open(ctx.attr("file_path"), "rb") as f:
        lt = S.read_lod_tensor(f, ctx.device)
    if ctx.attr("load_as_fp16"):
        lt = core.LoDTensor(lt.tensor.half(), lt.lod())
    ctx.set_output("Out", lt)


@register_op("save_combine", ["X*"], [], {"overwrite": True, "save_as_fp16": False, "file_path": ""}, grad=None,
             no_infer=True)
def save_combine(ctx):
    path = ctx.attr("file_path")
    if os.path.exists(path) and not ctx.attr("overwrite"):
        raise RuntimeError(f"{path} exists; set overwrite=True")
    _ensure_dir(path)
    with open(path, "wb") as f:
        for v in ctx.input_values("X"):
            if ctx.attr("save_as_fp16") and v.tensor.is_floating_point():
                v = core.LoDTensor(v.tensor.half(), v.lod())
            S.write_lod_tensor(f, v)


@register_op("load_combine", [], ["Out*"], {"file_path": "", "load_as_fp16": False}, grad=None, no_infer=True)
def load_combine(ctx):
    n = len(ctx.output_names("Out"))
    with open(ctx.attr("file_path"), "rb") as f:
        for i in range(n):
            lt = S.read_lod_tensor(f, ctx.device)
            if ctx.attr("load_as_fp16"):
                lt = core.LoDTensor(lt.tensor.half(), lt.lod())
            ctx.set_output("Out", lt, i=i)


# ------------------------------------------------------------------ control flow


def _cond_true(v):
    t = v.tensor if isinstance(v, core.LoDTensor) else v
    return bool(t.reshape(-1)[0].item()) if t.numel() else False


@register_op("while", ["X*", "Condition"], ["Out*", "StepScopes"], {"sub_block": None, "is_test": False},
             grad=None, no_infer=True, share_lod=False)
def while_op(ctx):
    """Runs sub_block in a child scope while Condition holds (while_op.cc)."""
    op, scope, exe = ctx.op, ctx.scope, ctx.executor
    blk = ctx.attr("sub_block")
    cond_name = op.input("Condition")[0]
    steps = []
    while _cond_true(scope.find_var(cond_name).get()):
        s = scope.new_scope()
        steps.append(s)
        exe.run_block(blk.program, blk.idx, s)
        # write back sub-block results visible to the parent (vars declared outside)
        for n in s.local_var_names():
            if blk.program.block(blk.parent_idx)._find_var_recursive(n) is not None:
                pv = scope.find_var(n)
                if pv is not None:
                    pv.set(s.find_local_var(n).get())
    if ctx.has_output("StepScopes"):
        ctx.set_output("StepScopes", steps)


@register_op("conditional_block", ["X*", "Cond*"], ["Out*", "Scope"],
             {"sub_block": None, "is_scalar_condition": False}, grad=None, no_infer=True, share_lod=False)
def conditional_block(ctx):
    op, scope, exe = ctx.op, ctx.scope, ctx.executor
    blk = ctx.attr("sub_block")
    conds = ctx.input_values("Cond")
    if ctx.attr("is_scalar_condition"):
        run = _cond_true(conds[0])
    else:
        run = all((c.tensor.numel() > 0) for c in conds if isinstance(c, core.LoDTensor))
    if not run:
        if ctx.has_output("Scope"):
            ctx.set_output("Scope", [])  # no kept scope: the grad op knows the block did not run
        return
    s = scope.new_scope()
    exe.run_block(blk.program, blk.idx, s)
    parent = blk.program.block(blk.parent_idx)
    for n in s.local_var_names():
        if parent._find_var_recursive(n) is not None:
            pv = scope.find_var(n) or scope.var(n)
            pv.set(s.find_local_var(n).get())
    if ctx.has_output("Scope"):
        ctx.set_output("Scope", [s])


# ------------------------------------------------------------------ tensor arrays & LoD rank tables


@register_op("write_to_array", ["X", "I"], ["Out"], {}, no_infer=True, share_lod=False)
def write_to_array(ctx):
    i = int(ctx.input("I").reshape(-1)[0].item())
    name = ctx.op.output("Out")[0]
    var = ctx.scope.find_var(name)
    arr = var.get() if var is not None and isinstance(var.get(), core.LoDTensorArray) else core.LoDTensorArray()
    while len(arr) <= i:
        arr.append(None)
    v = ctx.input_value("X")
    arr[i] = core.LoDTensor(v.tensor, v.lod()) if isinstance(v, core.LoDTensor) else v
    ctx.set_output("Out", arr)


@register_op("read_from_array", ["X", "I"], ["Out"], {}, no_infer=True, share_lod=False)
def read_from_array(ctx):
    arr = ctx.input_value("X")
    i = int(ctx.input("I").reshape(-1)[0].item())
    v = arr[i]
    ctx.set_output("Out", core.LoDTensor(v.tensor, v.lod()))


@register_op("lod_array_length", ["X"], ["Out"], {}, grad=None, no_infer=True)
def lod_array_length(ctx):
    ctx.set_output("Out", torch.tensor([len(ctx.input_value("X"))], dtype=torch.int64))


@register_op("lod_rank_table", ["X"], ["Out"], {"level": 0}, grad=None, no_infer=True, share_lod=False)
def lod_rank_table(ctx):
    """Sequences sorted by length, descending (lod_rank_table.cc)."""
    lod = ctx.input_lod("X")
    lvl = lod[ctx.attr("level")] if lod else [0, ctx.input("X").shape[0]]
    lens = [(i, lvl[i + 1] - lvl[i]) for i in range(len(lvl) - 1)]
    lens.sort(key=lambda x: -x[1])
    t = core.LoDRankTable(lens)
    t.coarse_lod = lod[:ctx.attr("level")]
    ctx.set_output("Out", t)


@register_op("max_sequence_len", ["RankTable"], ["Out"], {}, grad=None, no_infer=True)
def max_sequence_len(ctx):
    t = ctx.input_value("RankTable")
    ctx.set_output("Out", torch.tensor([t.items[0][1] if t.items else 0], dtype=torch.int64))


@register_op("lod_tensor_to_array", ["X", "RankTable"], ["Out"], {}, no_infer=True, share_lod=False)
def lod_tensor_to_array(ctx):
    """Time-major split: array[t] = rows at step t of every sequence still alive (sorted by rank)."""
    x = ctx.input("X")
    tab = ctx.input_value("RankTable")
    lod = ctx.input_lod("X")
    lvl = lod[-1] if lod else [0, x.shape[0]]
    arr = core.LoDTensorArray()
    maxlen = tab.items[0][1] if tab.items else 0
    for t in range(maxlen):
        idx = [lvl[i] + t for i, l in tab.items if l > t]
        arr.append(core.LoDTensor(x[torch.as_tensor(idx, device=x.device, dtype=torch.long)]))
    ctx.set_output("Out", arr)


@register_op("array_to_lod_tensor", ["X", "RankTable"], ["Out"], {}, no_infer=True, share_lod=False)
def array_to_lod_tensor(ctx):
    arr = ctx.input_value("X")
    tab = ctx.input_value("RankTable")
    n = len(tab.items)
    seqs = {i: [] for i, _ in tab.items}
    for t, lt in enumerate(arr):
        alive = [i for i, l in tab.items if l > t]
        for k, i in enumerate(alive):
            seqs[i].append(lt.tensor[k])
    order = sorted(seqs.keys())
    rows, off = [], [0]
    for i in order:
        rows += seqs[i]
        off.append(off[-1] + len(seqs[i]))
    out = torch.stack(rows) if rows else torch.zeros(0)
    ctx.set_output("Out", out, [off])


@register_op("shrink_rnn_memory", ["X", "I", "RankTable"], ["Out"], {}, no_infer=True, share_lod=False)
def shrink_rnn_memory(ctx):
    x = ctx.input("X")
    i = int(ctx.input("I").reshape(-1)[0].item())
    tab = ctx.input_value("RankTable")
    alive = sum(1 for _, l in tab.items if l > i)
    ctx.set_output("Out", x[:alive])


@register_op("reorder_lod_tensor_by_rank", ["X", "RankTable"], ["Out"], {}, no_infer=True, share_lod=False)
def reorder_lod_tensor_by_rank(ctx):
    x = ctx.input("X")
    tab = ctx.input_value("RankTable")
    lod = ctx.input_lod("X")
    if not lod:
        idx = [i for i, _ in tab.items]
        ctx.set_output("Out", x[torch.as_tensor(idx, dtype=torch.long, device=x.device)])
        return
    lvl = lod[0]
    rows, off = [], [0]
    for i, _ in tab.items:
        rows += list(range(lvl[i], lvl[i + 1]))
        off.append(off[-1] + lvl[i + 1] - lvl[i])
    ctx.set_output("Out", x[torch.as_tensor(rows, dtype=torch.long, device=x.device)], [off])


@register_op("split_lod_tensor", ["X", "Mask"], ["OutTrue", "OutFalse"], {"level": 0}, no_infer=True,
             share_lod=False)
def split_lod_tensor(ctx):
    x, m = ctx.input("X"), ctx.input("Mask").reshape(-1).bool()
    ctx.set_output("OutTrue", x[m])
    ctx.set_output("OutFalse", x[~m])


@register_op("merge_lod_tensor", ["X", "Mask", "InTrue", "InFalse"], ["Out"], {"level": 0}, no_infer=True,
             share_lod=False)
def merge_lod_tensor(ctx):
    m = ctx.input("Mask").reshape(-1).bool()
    t, f = ctx.input("InTrue"), ctx.input("InFalse")
    ref = t if t is not None and t.numel() else f
    out = torch.zeros((m.shape[0],) + tuple(ref.shape[1:]), dtype=ref.dtype, device=ref.device)
    if t is not None and t.numel():
        out[m] = t
    if f is not None and f.numel():
        out[~m] = f
    ctx.set_output("Out", out)


@register_op("get_places", [], ["Out"], {"device_count": 0, "device_type": "AUTO"}, grad=None, no_infer=True)
def get_places(ctx):
    n = ctx.attr("device_count") or max(1, core.get_cuda_device_count())
    if ctx.attr("device_type") == "CPU" or not core.is_compiled_with_cuda():
        ctx.set_output("Out", [core.CPUPlace() for _ in range(n)])
    else:
        ctx.set_output("Out", [core.CUDAPlace(i) for i in range(n)])


@register_op("rnn_memory_helper", ["X"], ["Out"], {"dtype": 5}, no_infer=True)
def rnn_memory_helper(ctx):
    v = ctx.input_value("X")
    ctx.set_output("Out", core.LoDTensor(v.tensor, v.lod()))
