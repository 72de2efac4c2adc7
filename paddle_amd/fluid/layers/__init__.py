"""paddle.fluid.layers."""
from . import control_flow, io, learning_rate_scheduler, math_op_patch, metric_op, nn, ops, tensor  # noqa: F401
from .control_flow import *  # noqa: F401,F403
from .io import *  # noqa: F401,F403
from .io import data  # noqa: F401
from .learning_rate_scheduler import *  # noqa: F401,F403
from .metric_op import *  # noqa: F401,F403
from .nn import *  # noqa: F401,F403
from .ops import *  # noqa: F401,F403
from .tensor import *  # noqa: F401,F403
from .sequence import *  # noqa: F401,F403
from .detection import *  # noqa: F401,F403
from . import rnn  # noqa: F401,E402
from .rnn import *  # noqa: F401,F403,E402
