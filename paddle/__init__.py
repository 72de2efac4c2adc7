"""``import paddle`` entry point: aliases of the paddle_amd framework so user code
written against the reference (``import paddle.fluid as fluid``, ``paddle.batch``,
``paddle.reader``, ``paddle.dataset``) runs unchanged on MI355X."""
import sys as _sys

import paddle_amd as _pa
from paddle_amd import fluid  # noqa: F401
from paddle_amd import reader  # noqa: F401
from paddle_amd import dataset  # noqa: F401
from paddle_amd.reader import batch  # noqa: F401

__version__ = _pa.__version__
_sys.modules[__name__ + ".fluid"] = fluid
_sys.modules[__name__ + ".reader"] = reader
_sys.modules[__name__ + ".dataset"] = dataset
for _k, _v in list(_sys.modules.items()):
    if _k.startswith("paddle_amd.fluid."):
        _sys.modules["paddle.fluid." + _k[len("paddle_amd.fluid."):]] = _v
