"""The control-flow / SelectedRows programs of test_native_engine_control_cpu.py on a
HIP place: while / while_grad step scopes, tensor arrays, rank tables and sparse
embedding gradients run on the device kernels (ops_gpu.hip, ops_control.cc) with
no Python-kernel fallback AND no host round trip (host_fallbacks == {}), following
the Python engine on the same device to 2e-4."""
import numpy as np
import pytest

import paddle_amd.fluid as fluid

from native_control_cases import CASES, run

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", sorted(CASES))
def test_control_program_native_matches_python_gpu(case):
    build, feeds = CASES[case]
    fd = feeds()
    place = fluid.CUDAPlace(0)
    ref, init, _ = run(build, fd, "python", place)
    got, _, exe = run(build, fd, "native", place, init=init)
    for r, g in zip(ref, got):
        for a, b in zip(r, g):
            np.testing.assert_allclose(b, a, rtol=2e-4, atol=2e-5)
    eng = exe._native
    assert not eng.py_fallbacks, eng.py_fallbacks
    assert not eng.host_fallbacks(), eng.host_fallbacks()


def test_device_ops_program_strict_native_gpu(monkeypatch):
    """FLAGS_strict_native makes a device-place host fallback an error: the program
    of formerly host-only ops runs entirely on device kernels."""
    from native_control_cases import CASES_DEVICE_OPS

    monkeypatch.setenv("FLAGS_strict_native", "1")
    build, feeds = CASES_DEVICE_OPS["device_ops"]
    fd = feeds()
    place = fluid.CUDAPlace(0)
    ref, init, _ = run(build, fd, "python", fluid.CPUPlace())
    got, _, exe = run(build, fd, "native", place, init=init)
    for r, g in zip(ref, got):
        for a, b in zip(r, g):
            np.testing.assert_allclose(np.asarray(b, dtype="float64"), np.asarray(a, dtype="float64"),
                                       rtol=2e-4, atol=2e-5)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks
    assert not exe._native.host_fallbacks(), exe._native.host_fallbacks()
