"""Liveness-based memory release (transpiler/memory_optimization_transpiler.py:47-400).

The reference renames variables so later temporaries reuse the buffers of dead
ones.  On MI355X the tensor storage comes from a caching allocator, so the same
effect is obtained by releasing each temporary right after its last use: a
``delete_var`` op is inserted there, the allocator then hands the block to the
next producer.  Persistables, feed/fetch targets and ``skip_opt_set`` are kept.
"""
from __future__ import annotations

from ...framework import core


def _liveness(block, skip):
    last_use = {}
    for i, op in enumerate(block.ops):
        for n in op.input_arg_names + op.output_arg_names:
            last_use[n] = i
    frees = {}
    for n, i in last_use.items():
        v = block._find_var_recursive(n)
        if v is None or v.persistable or n in skip or v.type not in (core.VT.LOD_TENSOR,):
            continue
        frees.setdefault(i, []).append(n)
    return frees


def memory_optimize(input_program, skip_opt_set=None, print_log=False, level=0, skip_grads=False):
    skip = set(skip_opt_set or [])
    block = input_program.global_block()
    for op in block.ops:
        if op.type in ("fetch", "feed"):
            skip.update(op.input_arg_names + op.output_arg_names)
        if op.type in ("while", "conditional_block", "recurrent"):
            return  # sub-block liveness not modelled: leave program unchanged
    frees = _liveness(block, skip)
    for i in sorted(frees.keys(), reverse=True):
        block.insert_op(i + 1, type="delete_var", inputs={"X": frees[i]}, outputs={})
    if print_log:
        print(f"memory_optimize: release points inserted for {sum(len(v) for v in frees.values())} vars")
    input_program._version += 1


def release_memory(input_program, skip_opt_set=None):
    memory_optimize(input_program, skip_opt_set)
