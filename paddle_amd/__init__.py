"""paddle_amd -- a PaddlePaddle-compatible deep-learning framework written for
AMD Instinct MI355X (CDNA4 / gfx950).

Layers (see SURVEY.md §1 for the reference's layer map):
  * ``paddle_amd.ops``       hand-written gfx950 HIP kernels (+ CPU reference kernels)
  * ``paddle_amd.framework`` Program/Block/Operator IR, Scope, Executor (static graph)
  * ``paddle_amd.fluid``     the ``paddle.fluid`` Python API
  * ``paddle_amd.dygraph`` / ``paddle_amd.nn``  eager (DyGraph) layers on the same kernels
  * ``paddle_amd.parallel``  RCCL-over-xGMI data/tensor/pipeline/sharding/expert parallelism
  * ``paddle_amd.models``    LLaMA, GPT, ERNIE-MoE, ResNet, LeNet, Transformer
  * ``paddle_amd.utils``     flags, profiler, checkpoint helpers
"""
import torch  # noqa: F401  (loads the HIP runtime our kernel library links against)

__version__ = "0.1.0"

from . import ops  # noqa: E402,F401
