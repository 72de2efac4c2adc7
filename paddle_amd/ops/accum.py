"""Deferred weight-gradient work across the micro-batches of one optimizer step.

Gradient accumulation runs the backward once per micro-batch; a weight gradient
that accumulates into an fp32 main_grad then pays a read-modify-write of that
main_grad per micro-batch.  While :func:`deferring` is true (the sharded
optimizers' ``no_sync()`` -- every micro-batch but the last) an op may keep the
operands of its weight gradient instead and compute it once, over all micro-batches,
in the last one (``ops/grouped.py``: the experts' dW as one grouped GEMM whose K is
every micro-batch's tokens, one main_grad write per step).  :func:`flush` computes
whatever is still pending (called by the optimizer step before it reads main_grad).

Memory: a deferring op keeps its dW operands alive until the last micro-batch -- for
the MoE experts x / dh / a / dy of every deferred micro-batch of every MoE layer (at
most ``_MAX_MB - 1`` = 7 per layer; ``FLAGS_defer_expert_wgrad=0`` turns deferral off).
:func:`discard` drops pending work unused: ``zero_grad`` / ``clear_grad`` (the step
was abandoned, e.g. an AMP inf/nan skip) and a ``no_sync`` block that raised, so
stale operands never reach the next step's main_grad.

Reference counterpart: Fleet's gradient merge (``accumulate_steps``) sums per
micro-batch gradients; the sum is the same, the order of the additions differs.
"""
from __future__ import annotations

_STATE = {"defer": False}
_FLUSH = []
_DISCARD = []


def deferring() -> bool:
    return _STATE["defer"]


def set_deferring(on: bool) -> None:
    _STATE["defer"] = bool(on)


def register_flush(fn) -> None:
    if fn not in _FLUSH:
        _FLUSH.append(fn)


def flush() -> None:
    """Compute every deferred weight gradient now (before main_grad is read)."""
    for fn in _FLUSH:
        fn()


def register_discard(fn) -> None:
    if fn not in _DISCARD:
        _DISCARD.append(fn)


def discard() -> None:
    """Drop every deferred weight gradient without computing it (the accumulated
    step was abandoned: zero_grad / clear_grad, or an exception inside no_sync)."""
    for fn in _DISCARD:
        fn()
