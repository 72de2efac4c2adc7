"""``paddle.v2``: the reference's legacy v2 training API (python/paddle/v2:
``init``, ``layer``, ``data_type``, ``activation``, ``pooling``, ``attr``,
``networks``, ``optimizer``, ``parameters``, ``trainer.SGD`` with events,
``evaluator``, ``topology``, ``infer``) re-implemented as a facade over this
framework's Fluid programs and executors -- v2 topologies become one Fluid
program, ``trainer.SGD.train`` drives the Fluid executor (HIP kernels on the
GPU), and parameters keep the v2 tar format (per-parameter 16-byte header +
raw float32 values).  The SWIG GradientMachine behind the reference
implementation is not carried over (SURVEY §7 non-goal)."""
from . import activation, attr, data_type, evaluator, event, inference, layer, networks, optimizer  # noqa: F401
from . import parameters, pooling, topology, trainer  # noqa: F401
from ._core import STATE as _STATE
from ._core import reset as _reset
from .inference import infer  # noqa: F401

__all__ = ["optimizer", "layer", "activation", "parameters", "init", "trainer", "event", "data_type", "attr",
           "pooling", "topology", "networks", "infer", "evaluator"]


def init(use_gpu=False, trainer_count=1, **kwargs):
    """Start a fresh v2 session (reference v2/__init__.py ``init``): picks the
    place; ``trainer_count`` > 1 is accepted (the Fluid executor uses the whole
    device)."""
    _reset()
    _STATE["use_gpu"] = bool(use_gpu)
    _STATE["trainer_count"] = int(trainer_count)
    _STATE["init"] = True
