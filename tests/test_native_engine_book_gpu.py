"""The book programs on the C++ executor with a HIP place: device kernels
(ops_gpu.hip) on torch's current stream, host kernels for the rest, and the
while sub-block run by Executor::RunWhile -- the trajectory must match the Python
engine on the same device."""
import numpy as np
import pytest

import paddle_amd.fluid as fluid

from test_native_engine_book_cpu import CASES, _run

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", sorted(CASES))
def test_book_program_native_matches_python_gpu(case):
    build, feeds = CASES[case]
    fd = feeds()
    place = fluid.CUDAPlace(0)
    ref, init, _ = _run(build, fd, "python", place)
    got, _, exe = _run(build, fd, "native", place, init=init)
    for r, g in zip(ref, got):
        for a, b in zip(r, g):
            np.testing.assert_allclose(b, a, rtol=2e-4, atol=2e-5)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks
