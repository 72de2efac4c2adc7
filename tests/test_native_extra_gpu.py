"""ops_extra.hip and the transposed convolutions on a HIP place: the cases of
test_native_extra_cpu.py on the C++ executor's device kernels vs the interpreter,
no Python or host fallback."""
import pytest

import paddle_amd.fluid as fluid

from test_native_extra_cpu import BUILDS, check

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", sorted(BUILDS))
def test_extra_op_native_gpu(case):
    exe = check(case, fluid.CUDAPlace(0), 2e-4, 2e-5)
    assert not exe._native.host_fallbacks(), exe._native.host_fallbacks()
