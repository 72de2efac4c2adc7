"""paddle.optimizer (DyGraph) -- fused gfx950 update kernels for Adam/AdamW/Momentum/SGD."""
from . import lr  # noqa: F401
from .clip import ClipGradByGlobalNorm, ClipGradByNorm, ClipGradByValue  # noqa: F401
from .optimizer import (SGD, Adadelta, Adagrad, Adam, Adamax, AdamW, L1Decay, L2Decay, Lamb,  # noqa: F401
                        Momentum, Optimizer, RMSProp)
