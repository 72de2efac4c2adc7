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


def test_fusion_rnn_native_gpu():
    from native_control_cases import run
    from test_native_extra_cpu import fusion_feeds, fusion_rnn_build
    import numpy as np
    place = fluid.CUDAPlace(0)
    ref, init, _ = run(fusion_rnn_build, fusion_feeds(), "python", place)
    got, _, exe = run(fusion_rnn_build, fusion_feeds(), "native", place, init)
    for u, v in zip(ref[0], got[0]):
        np.testing.assert_allclose(v, u, rtol=2e-4, atol=2e-5)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks
    assert not exe._native.host_fallbacks(), exe._native.host_fallbacks()
