"""``import paddle`` entry point: aliases of the paddle_amd framework so user code
written against Paddle -- the 1.x static API (``import paddle.fluid as fluid``,
``paddle.batch``, ``paddle.reader``, ``paddle.dataset``) and the 2.x DyGraph API
(``paddle.to_tensor``, ``paddle.nn``, ``paddle.optimizer``, ``paddle.io``,
``paddle.distributed.fleet``, ``paddle.save``/``load``) -- runs unchanged on MI355X."""
import sys as _sys

import paddle_amd as _pa
from paddle_amd import *  # noqa: F401,F403
from paddle_amd import (amp, checkpoint, distributed, io, metric, nn, optimizer, vision)  # noqa: F401
from paddle_amd import fluid  # noqa: F401
from paddle_amd import reader  # noqa: F401
from paddle_amd import dataset  # noqa: F401
from paddle_amd import dygraph  # noqa: F401
from paddle_amd import v2  # noqa: F401
from paddle_amd import trainer_config_helpers  # noqa: F401
from paddle_amd import trainer  # noqa: F401
from paddle_amd.reader import batch  # noqa: F401
from paddle_amd.checkpoint import load, save  # noqa: F401
from paddle_amd.hapi import Model  # noqa: F401

for _n in dir(_pa._tensor_api):
    if not _n.startswith("_") and _n not in ("annotations", "builtins", "math", "np", "torch"):
        globals()[_n] = getattr(_pa._tensor_api, _n)

static = fluid
__version__ = _pa.__version__
for _name, _mod in (("fluid", fluid), ("reader", reader), ("dataset", dataset), ("nn", nn),
                    ("optimizer", optimizer), ("io", io), ("amp", amp), ("metric", metric), ("vision", vision),
                    ("distributed", distributed), ("static", fluid), ("dygraph", dygraph),
                    ("v2", v2), ("trainer_config_helpers", trainer_config_helpers),
                    ("trainer", trainer), ("trainer.PyDataProvider2", trainer.PyDataProvider2)):
    _sys.modules[__name__ + "." + _name] = _mod
for _k, _v in list(_sys.modules.items()):
    for _src, _dst in (("paddle_amd.fluid.", "paddle.fluid."), ("paddle_amd.nn.", "paddle.nn."),
                       ("paddle_amd.distributed.", "paddle.distributed."), ("paddle_amd.optimizer.",
                                                                            "paddle.optimizer."),
                       ("paddle_amd.vision.", "paddle.vision."), ("paddle_amd.v2.", "paddle.v2.")):
        if _k.startswith(_src):
            _sys.modules[_dst + _k[len(_src):]] = _v
