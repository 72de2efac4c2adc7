"""paddle.nn: DyGraph layers on the gfx950 kernel library."""
from . import functional, initializer  # noqa: F401
from .layer import (Dropout, Embedding, Layer, LayerList, LayerNorm, Linear, RMSNorm,  # noqa: F401
                    Sequential)
from .layers_common import *  # noqa: F401,F403
from .layers_common import __all__ as _common_all
from .transformer import (GRU, LSTM, GRUCell, LSTMCell, MultiHeadAttention, SimpleRNN,  # noqa: F401
                          SimpleRNNCell, Transformer, TransformerDecoder, TransformerDecoderLayer,
                          TransformerEncoder, TransformerEncoderLayer)
from ..optimizer.clip import ClipGradByGlobalNorm, ClipGradByNorm, ClipGradByValue  # noqa: F401,E402
from . import utils  # noqa: F401,E402

Dropout2D = Dropout


def layer_bn_types():
    """BatchNorm layer classes (for fused BN+activation fast paths)."""
    from .layers_common import _BatchNormBase

    return (_BatchNormBase,)
