"""C++ lstm / gru kernels (csrc/native/ops_rnn.cc) on the native engine vs the Python
interpreter: same trajectory to 1e-5, and the recurrent ops (forward and grad) never
fall back to the Python op library."""
import numpy as np
import pytest

import paddle_amd.fluid as fluid

from native_control_cases import run
from native_rnn_cases import CASES, feeds


@pytest.mark.parametrize("case", sorted(CASES))
def test_native_rnn_matches_interpreter(case):
    build, kw = CASES[case]
    fd = feeds(4, **kw)
    place = fluid.CPUPlace()
    ref, init, _ = run(build, fd, "python", place)
    got, _, exe = run(build, fd, "native", place, init)
    for a, b in zip(ref, got):
        np.testing.assert_allclose(b[0], a[0], rtol=1e-5, atol=1e-6)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks
