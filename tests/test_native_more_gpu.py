"""ops_more.hip on a HIP place: the cases of test_native_more_cpu.py on the C++
executor's device kernels vs the interpreter, no Python or host fallback."""
import numpy as np
import pytest

import paddle_amd.fluid as fluid

from native_control_cases import run
from test_native_more_cpu import BUILDS, feeds

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", sorted(BUILDS))
def test_more_op_native_gpu(case):
    fd = feeds()
    place = fluid.CUDAPlace(0)
    ref, init, _ = run(BUILDS[case], fd, "python", place)
    got, _, exe = run(BUILDS[case], fd, "native", place, init)
    for a, b in zip(ref, got):
        np.testing.assert_allclose(b[0], a[0], rtol=2e-4, atol=2e-5)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks
    assert not exe._native.host_fallbacks(), exe._native.host_fallbacks()
