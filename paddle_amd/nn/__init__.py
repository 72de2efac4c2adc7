"""paddle.nn-style DyGraph layers on the gfx950 kernel library."""
from . import initializer  # noqa: F401
from .layer import (Dropout, Embedding, Layer, LayerList, LayerNorm, Linear, RMSNorm,  # noqa: F401
                    Sequential)
