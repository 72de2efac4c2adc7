"""Program transpilers (python/paddle/fluid/transpiler)."""
from .distribute_transpiler import DistributeTranspiler, DistributeTranspilerConfig  # noqa: F401
from .inference_transpiler import InferenceTranspiler  # noqa: F401
from .memory_optimization_transpiler import memory_optimize, release_memory  # noqa: F401
from .ps_dispatcher import HashName, RoundRobin  # noqa: F401
from .float16_transpiler import BF16Transpiler, Float16Transpiler, ReducedPrecisionTranspiler  # noqa: F401,E402
