"""Program pretty-printer and block graph dump for debugging (API of
python/paddle/fluid/debugger.py, written from its documented behaviour).

``pprint_program_codes(program)`` renders every block as pseudo-code::

    // block-0  parent--1
    // variables
    var fc_0.w_0 : LOD_TENSOR.shape(784, 200).astype(FP32) [persistable]
    // operators
    fc_0.tmp_0 = mul(X=img, Y=fc_0.w_0) [{x_num_col_dims=1,y_num_col_dims=1}]

backward variables / ops (``@GRAD`` names, ``*_grad`` ops) are hidden unless
``show_backward``.  ``draw_block_graphviz(block, highlights, path)`` writes a
graphviz dot file of the block's ops and variables; variable names matching any
regex in ``highlights`` are drawn in red.
"""
from __future__ import annotations

import re

from ..framework import core


def _vt_name(t):
    for k in dir(core.VT):
        if not k.startswith("_") and getattr(core.VT, k) == t:
            return k
    return str(t)


def repr_data_type(dtype):
    return _vt_name(dtype) if isinstance(dtype, int) else str(dtype).upper()


def repr_var(var):
    shape = tuple(var.shape) if getattr(var, "shape", None) is not None else ()
    dt = repr_data_type(var.dtype) if getattr(var, "dtype", None) is not None else "?"
    s = f"var {var.name} : {_vt_name(var.type)}.shape{shape}.astype({dt})"
    if getattr(var, "lod_level", 0):
        s += f".lod_level({var.lod_level})"
    if var.persistable:
        s += " [persistable]"
    return s


def repr_attr(key, value):
    if hasattr(value, "idx") and hasattr(value, "ops"):
        value = f"block[{value.idx}]"
    return f"{key}={value}"


def _arg(names):
    return names[0] if len(names) == 1 else str(list(names))


def repr_op(op):
    if op.type == "fill_constant":
        return f"{', '.join(op.output_arg_names)} = {op.attrs.get('value')} [shape={list(op.attrs.get('shape', []))}]"
    ins = ", ".join(f"{slot}={_arg(names)}" for slot, names in op.inputs.items() if names)
    outs = ", ".join(_arg(names) for names in op.outputs.values() if names)
    attrs = ",".join(repr_attr(k, v) for k, v in sorted(op.attrs.items()) if not k.startswith("op_"))
    return f"{outs} = {op.type}({ins}) [{{{attrs}}}]"


def _is_backward_op(op):
    if op.type.endswith("_grad"):
        return True
    return any("@GRAD" in n for n in op.input_arg_names + op.output_arg_names)


def pprint_block_codes(block, show_backward=False):
    vars_ = [repr_var(v) for v in block.vars.values() if show_backward or "@GRAD" not in v.name]
    ops = [repr_op(op) for op in block.ops if show_backward or not _is_backward_op(op)]
    return (f"// block-{block.idx}  parent-{block.parent_idx}\n// variables\n" + "\n".join(vars_) +
            "\n\n// operators\n" + "\n".join(ops) + "\n")


def pprint_program_codes(program, show_backward=False):
    return "\n".join(pprint_block_codes(b, show_backward) for b in program.blocks)


def draw_block_graphviz(block, highlights=None, path="./temp.dot"):
    """Write a dot graph of ``block`` (ops: boxes; vars: ellipses, parameters
    filled; names matching a ``highlights`` regex: red) and return its text."""
    pats = [re.compile(p) for p in (highlights or [])]
    lines = ["digraph G {", '  rankdir=TB; node [fontsize=10];']
    vid = {}

    def var_node(name):
        if name not in vid:
            vid[name] = f"v{len(vid)}"
            v = block._find_var_recursive(name)
            style = 'style=filled, fillcolor="#f0e6d2"' if v is not None and v.persistable else ""
            color = ", color=red, fontcolor=red" if any(p.match(name) for p in pats) else ""
            lines.append(f'  {vid[name]} [label="{name}", shape=ellipse {("," + style) if style else ""}{color}];')
        return vid[name]

    for i, op in enumerate(block.ops):
        on = f"o{i}"
        lines.append(f'  {on} [label="{op.type}", shape=box, style=filled, fillcolor="#dfe8f6"];')
        for n in op.input_arg_names:
            lines.append(f"  {var_node(n)} -> {on};")
        for n in op.output_arg_names:
            lines.append(f"  {on} -> {var_node(n)};")
    lines.append("}")
    dot = "\n".join(lines)
    if path:
        with open(path, "w") as f:
            f.write(dot)
    return dot
