"""SRL (book label_semantic_roles) from ONE set of initial parameters on the four
(engine, place) combinations: per-step losses, to tell which GPU engine diverges."""
import os
import sys

import numpy as np

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _ROOT)
sys.path.insert(0, os.path.join(_ROOT, "tests"))
import paddle_amd.fluid as fluid  # noqa: E402
from native_control_cases import run  # noqa: E402
from native_rnn_cases import srl, srl_feeds  # noqa: E402

fd = srl_feeds(3)
_, init, _ = run(srl(), fd[:1], "python", fluid.CUDAPlace(0))
init = {k: v.copy() for k, v in init.items()}
for eng, place in (("python", fluid.CPUPlace()), ("native", fluid.CPUPlace()), ("native", fluid.CUDAPlace(0)),
                   ("python", fluid.CUDAPlace(0))):
    got, _, _ = run(srl(), fd, eng, place, {k: v.copy() for k, v in init.items()})
    print(eng, type(place).__name__, [float(np.asarray(g[0]).ravel()[0]) for g in got], flush=True)
