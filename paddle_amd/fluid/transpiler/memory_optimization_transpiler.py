"""Liveness-based memory release (transpiler/memory_optimization_transpiler.py:47-400).

The reference renames variables so later temporaries reuse the buffers of dead
ones.  On MI355X the tensor storage comes from a caching allocator, so the same
effect is obtained by releasing each temporary right after its last use: a
``delete_var`` op is inserted there, the allocator then hands the block to the
next producer.  Persistables, feed/fetch targets and ``skip_opt_set`` are kept.

Control flow (the reference's ``ControlFlowGraph`` over sub-blocks, :381): an op
that owns a sub-block (while / conditional_block / recurrent / parallel_do) USES
every parent-scope variable its sub-blocks touch, so nothing the loop reads is
freed before the loop ends.  Inside a sub-block, temporaries declared there are
freed after their last use in the body when they are written before they are
read (not loop-carried) -- unless a ``*_grad`` op of that sub-block exists, whose
backward replays the forward step scopes.
"""
from __future__ import annotations

from ...framework import core

_CF_OPS = ("while", "conditional_block", "recurrent", "parallel_do")


def _sub_block(op, program):
    sb = op.attrs.get("sub_block")
    if sb is None:
        return None
    return sb if hasattr(sb, "ops") else program.block(int(sb))


def _block_refs(block, program):
    """All variable names an op list touches, sub-blocks included."""
    names = set()
    for op in block.ops:
        names.update(op.input_arg_names)
        names.update(op.output_arg_names)
        sb = _sub_block(op, program)
        if sb is not None:
            names |= _block_refs(sb, program)
    return names


def _op_uses(op, program):
    uses = set(op.input_arg_names) | set(op.output_arg_names)
    sb = _sub_block(op, program)
    if sb is not None:
        uses |= _block_refs(sb, program)
    return uses


def _freeable(block, n, skip, local_only):
    v = block.vars.get(n) if local_only else block._find_var_recursive(n)
    return v is not None and not v.persistable and n not in skip and v.type == core.VT.LOD_TENSOR


def _liveness(block, skip, program, local_only=False):
    last_use = {}
    for i, op in enumerate(block.ops):
        for n in _op_uses(op, program):
            last_use[n] = i
    frees = {}
    for n, i in last_use.items():
        if _freeable(block, n, skip, local_only):
            frees.setdefault(i, []).append(n)
    return frees


def _not_loop_carried(block, names, program):
    """Names first WRITTEN before any read in the body (so an iteration never sees
    the previous iteration's value)."""
    seen_w, carried = set(), set()
    for op in block.ops:
        reads = set(op.input_arg_names)
        sb = _sub_block(op, program)
        if sb is not None:
            reads |= _block_refs(sb, program)
        for n in reads:
            if n not in seen_w:
                carried.add(n)
        seen_w.update(op.output_arg_names)
    return [n for n in names if n not in carried]


def _insert_frees(block, frees):
    for i in sorted(frees.keys(), reverse=True):
        if frees[i]:
            block.insert_op(i + 1, type="delete_var", inputs={"X": frees[i]}, outputs={})


def memory_optimize(input_program, skip_opt_set=None, print_log=False, level=0, skip_grads=False):
    skip = set(skip_opt_set or [])
    program = input_program
    gb = program.global_block()
    for op in gb.ops:
        if op.type in ("fetch", "feed"):
            skip.update(op.input_arg_names + op.output_arg_names)
    grad_owned = set()  # sub-blocks whose forward step scopes a *_grad op replays
    for blk in program.blocks:
        for op in blk.ops:
            if op.type.endswith("_grad") and op.type[:-5] in _CF_OPS:
                sb = _sub_block(op, program)
                if sb is not None:
                    grad_owned.add(sb.idx)
                fwd_sb = op.attrs.get("original_sub_block") or op.attrs.get("fwd_sub_block")
                if fwd_sb is not None:
                    grad_owned.add(int(fwd_sb) if not hasattr(fwd_sb, "idx") else fwd_sb.idx)
    # forward sub-blocks of a while whose gradient exists are replayed: keep them whole
    for blk in program.blocks:
        for op in blk.ops:
            if op.type in _CF_OPS and any(o.type == op.type + "_grad" for b in program.blocks for o in b.ops):
                sb = _sub_block(op, program)
                if sb is not None:
                    grad_owned.add(sb.idx)
    total = 0
    frees = _liveness(gb, skip, program)
    total += sum(len(v) for v in frees.values())
    _insert_frees(gb, frees)
    for blk in program.blocks[1:]:
        if blk.idx in grad_owned:
            continue
        sub = _liveness(blk, skip, program, local_only=True)
        for i in list(sub):
            sub[i] = _not_loop_carried(blk, sub[i], program)
        total += sum(len(v) for v in sub.values())
        _insert_frees(blk, sub)
    if print_log:
        print(f"memory_optimize: release points inserted for {total} vars")
    input_program._version += 1
    return total


def release_memory(input_program, skip_opt_set=None):
    memory_optimize(input_program, skip_opt_set)
