"""Shared state of the v2 facade: one Fluid program pair + scope that every v2
layer call appends to (the reference v2 API parses a model config into one
topology; here that topology IS a Fluid program), the run place chosen by
``paddle.v2.init``, and the side tables v2 needs (data-layer types, layer sizes)."""
from __future__ import annotations

from .. import fluid

STATE = {"main": fluid.Program(), "startup": fluid.Program(), "scope": fluid.core.Scope(), "use_gpu": False,
         "data": {}, "init": False}


def reset():
    STATE.update(main=fluid.Program(), startup=fluid.Program(), scope=fluid.core.Scope(), data={}, evaluators=[])


def guard():
    return fluid.program_guard(STATE["main"], STATE["startup"])


def place():
    import torch

    if STATE["use_gpu"] and torch.cuda.is_available():
        return fluid.CUDAPlace(0)
    return fluid.CPUPlace()


def executor():
    return fluid.Executor(place())
