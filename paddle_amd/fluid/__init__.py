"""paddle.fluid -- the static-graph (Program/Executor) API on MI355X.

API surface follows paddle/fluid/API.spec of the reference; programs are built
in Python, serialised with the wire-compatible framework.proto schema, and run by
the block interpreter over gfx950 HIP kernels.
"""
from .. import operators as _operators  # noqa: F401  (registers all op kernels)
from ..framework import core  # noqa: F401
from ..framework.core import (CPUPlace, CUDAPinnedPlace, CUDAPlace, LoDTensor, LoDTensorArray, Scope,  # noqa: F401
                              Tensor)
from . import (backward, clip, data_feeder, executor, framework, initializer, io, layers, nets,  # noqa: F401
               optimizer, param_attr, profiler, regularizer, unique_name)
from .backward import append_backward, calc_gradient, gradients  # noqa: F401
from . import concurrency  # noqa: F401,E402
from .concurrency import Go, Select, channel_close, channel_recv, channel_send, make_channel  # noqa: F401,E402
from .data_feeder import DataFeeder  # noqa: F401
from .executor import Executor, global_scope, scope_guard  # noqa: F401
from .framework import (Operator, Parameter, Program, Variable, default_main_program,  # noqa: F401
                        default_startup_program, get_var, name_scope, program_guard)
from .initializer import init_on_cpu  # noqa: F401
from .lod_tensor import create_lod_tensor, create_random_int_lodtensor  # noqa: F401
from .param_attr import ParamAttr, WeightNormParamAttr  # noqa: F401
from .parallel_executor import BuildStrategy, ExecutionStrategy, ParallelExecutor  # noqa: F401
from .layers.math_op_patch import monkey_patch_variable

HIPPlace = CUDAPlace
Tensor = LoDTensor

monkey_patch_variable()

from . import metrics, average, evaluator, transpiler, contrib, recordio_writer, trainer, inferencer  # noqa: E402,F401
from .transpiler import (DistributeTranspiler, DistributeTranspilerConfig, InferenceTranspiler,  # noqa: E402,F401
                         memory_optimize, release_memory)
from .trainer import (BeginEpochEvent, BeginStepEvent, CheckpointConfig, EndEpochEvent, EndStepEvent,  # noqa: E402,F401
                      Trainer)
from .inferencer import Inferencer  # noqa: E402,F401
from ..utils.flags import init_gflags as _init_gflags  # noqa: E402


def __bootstrap__():
    """Mirror of the reference's bootstrap: read FLAGS_* from env (fluid/__init__.py:92-146)."""
    import os

    read_env_flags = ["use_pinned_memory", "check_nan_inf", "benchmark", "eager_delete_scope", "use_mkldnn",
                      "initial_cpu_memory_in_mb", "init_allocated_mem", "free_idle_memory", "paddle_num_threads",
                      "dist_threadpool_size", "cpu_deterministic", "fraction_of_gpu_memory_to_use",
                      "cudnn_deterministic", "allocator_strategy", "use_hip_graph", "rccl_bucket_mb"]
    _init_gflags(["--tryfromenv=" + ",".join(read_env_flags)])
    os.environ.setdefault("OMP_NUM_THREADS", "1")


__bootstrap__()
