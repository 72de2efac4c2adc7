"""paddle_amd -- a PaddlePaddle-compatible deep-learning framework written for
AMD Instinct MI355X (CDNA4 / gfx950).

Layers (see SURVEY.md §1 for the reference's layer map):
  * ``paddle_amd.ops``        hand-written gfx950 HIP kernels (+ CPU reference kernels)
  * ``paddle_amd.framework``  Program/Block/Operator IR, Scope, Executor (static graph)
  * ``paddle_amd.fluid``      the ``paddle.fluid`` (1.x static-graph) Python API
  * ``paddle_amd.nn`` / ``optimizer`` / ``io`` / ``amp`` / ``metric`` / ``vision``
                              the ``paddle.*`` 2.x DyGraph API on the same kernels
  * ``paddle_amd.distributed`` RCCL-over-xGMI DP / Fleet TP / PP / sharding / EP / CP
  * ``paddle_amd.models``     LLaMA, GPT, ERNIE-MoE model families
  * ``paddle_amd.runtime``    native C++ runtime (RecordIO, allocator, queues, scheduler)
"""
import torch  # noqa: F401  (loads the HIP runtime our kernel library links against)

__version__ = "0.1.0"


def _install_allocator():
    """FLAGS_allocator_strategy (default ``buddy``): torch's device tensors come from
    the native buddy allocator (csrc/runtime/allocator.cc; reference
    memory/detail/buddy_allocator.cc), with record_stream-ordered frees.  Any other
    value (``naive_best_fit``, ``auto_growth``, ``torch``) keeps torch's caching
    allocator.  It has to be swapped in before the first device allocation, hence at
    import; devices are counted without initialising HIP."""
    import os
    import warnings

    if os.environ.get("FLAGS_allocator_strategy", "buddy") != "buddy":
        return
    try:
        if torch.cuda.device_count() == 0:
            return
        from . import runtime

        mb = int(os.environ.get("FLAGS_buddy_chunk_mb", "4096"))
        runtime.use_buddy_allocator_for_torch(chunk_bytes=mb << 20)
    except Exception as e:  # noqa: BLE001  (torch already allocated on the device, lib missing, ...)
        warnings.warn(f"paddle_amd: buddy allocator not installed ({e}); using torch's caching allocator")


def _install_device_tracer():
    """FLAGS_device_tracer=1 (or PADDLE_AMD_DEVICE_TRACER=1): register the
    rocprofiler-sdk kernel tracer (utils/device_tracer.py) now, before anything
    initialises the HIP runtime."""
    import os

    on = os.environ.get("PADDLE_AMD_DEVICE_TRACER", os.environ.get("FLAGS_device_tracer", "0"))
    if on.lower() in ("1", "true", "yes"):
        from .utils import device_tracer

        if not device_tracer.install():
            import warnings

            warnings.warn(f"paddle_amd: device tracer not installed ({device_tracer.error()})")


_install_device_tracer()
_install_allocator()

from . import ops  # noqa: E402,F401
from . import tensor_api as _tensor_api  # noqa: E402

for _n in dir(_tensor_api):
    if not _n.startswith("_") and _n not in ("annotations", "builtins", "math", "np", "torch"):
        globals()[_n] = getattr(_tensor_api, _n)
Tensor = _tensor_api.Tensor

from . import amp, io, metric, nn, optimizer  # noqa: E402,F401
from . import distributed  # noqa: E402,F401
from . import vision  # noqa: E402,F401
from .checkpoint import load, save  # noqa: E402,F401
from .hapi import Model  # noqa: E402,F401
from .nn.layer import Layer  # noqa: E402,F401
from .framework.core import CPUPlace, CUDAPinnedPlace, CUDAPlace  # noqa: E402,F401

ParamAttr = None  # set lazily from fluid (avoids importing the static stack eagerly)

float32, float64, float16, bfloat16 = "float32", "float64", "float16", "bfloat16"
int8, int16, int32, int64, uint8, bool_ = "int8", "int16", "int32", "int64", "uint8", "bool"
HIPPlace = CUDAPlace


def disable_static(place=None):
    from . import dygraph

    dygraph.enable_dygraph(place)


def enable_static():
    from . import dygraph

    dygraph.disable_dygraph()


def in_dynamic_mode():
    return True


def __getattr__(name):
    if name in ("fluid", "static", "dygraph", "jit", "models", "runtime", "reader", "dataset", "hapi", "utils",
                "framework", "inference"):
        import importlib

        mod = importlib.import_module(f".{'fluid' if name == 'static' else name}", __name__)
        globals()[name] = mod
        return mod
    if name == "ParamAttr":
        from .fluid.param_attr import ParamAttr as PA

        return PA
    raise AttributeError(name)
