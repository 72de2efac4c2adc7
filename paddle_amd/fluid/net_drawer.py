"""Graphviz drawing of a training program pair (API of
python/paddle/fluid/net_drawer.py): ``draw_graph(startup_program, main_program,
**kwargs)`` returns the dot source of the startup and main programs' global blocks
as two clusters (ops as boxes, variables as ellipses, parameters highlighted) and
writes it to ``kwargs["filename"]`` when given.  No graphviz binary is needed to
produce the text; render it with ``dot -Tpng`` where available.
"""
from __future__ import annotations

import itertools

_ids = itertools.count()


def unique_id():
    return f"n{next(_ids)}"


def draw_node(op):
    return f'[label="{op.type}", shape=box, style="rounded,filled", fillcolor="#dfe8f6"]'


def draw_edge(src, dst, label=""):
    attr = ' [label="%s"]' % label if label else ""
    return f"  {src} -> {dst}{attr};"


def parse_graph(program, lines, var_dict, prefix=""):
    block = program.global_block()
    for op in block.ops:
        oid = unique_id()
        lines.append(f"  {oid} {draw_node(op)};")
        for slot, names in op.inputs.items():
            for n in names:
                if n not in var_dict:
                    var_dict[n] = unique_id()
                    v = block._find_var_recursive(n)
                    fill = ', style=filled, fillcolor="#f0e6d2"' if v is not None and v.persistable else ""
                    lines.append(f'  {var_dict[n]} [label="{n}", shape=ellipse{fill}];')
                lines.append(draw_edge(var_dict[n], oid, slot))
        for slot, names in op.outputs.items():
            for n in names:
                if n not in var_dict:
                    var_dict[n] = unique_id()
                    lines.append(f'  {var_dict[n]} [label="{n}", shape=ellipse];')
                lines.append(draw_edge(oid, var_dict[n], slot))


def draw_graph(startup_program, main_program, **kwargs):
    lines = ["digraph G {", "  rankdir=TB; node [fontsize=10];"]
    var_dict = {}
    for label, prog in (("startup", startup_program), ("main", main_program)):
        if prog is None:
            continue
        lines.append(f"  subgraph cluster_{label} {{ label=\"{label}\";")
        parse_graph(prog, lines, var_dict)
        lines.append("  }")
    lines.append("}")
    dot = "\n".join(lines)
    fn = kwargs.get("filename")
    if fn:
        with open(fn, "w") as f:
            f.write(dot)
    return dot
