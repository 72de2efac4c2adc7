"""fluid.Executor(CUDAPlace, engine="native") on MI355X: the C++ executor's device
kernels (ops_gpu.hip on the shared kernel library: pa_sgemm conv / GEMM, pa_pool,
pa_bn_nchw, pa_act, softmax / cross-entropy, pa_adamw / pa_momentum) train LeNet
and a ResNet-tiny along the Python executor's trajectory with every op on the
device (no host fallback).

Reference: framework/executor.cc:125-353, pybind/pybind.cc:507."""
import os

import numpy as np
import pytest

import paddle_amd.fluid as fluid
from native_engine_cases import train

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("model", ["lenet", "resnet_tiny"])
def test_native_engine_matches_python_trajectory_gpu(model):
    place = fluid.CUDAPlace(0)
    ref, ref_p, init, _ = train(model, place, "python", steps=5)
    got, got_p, _, exe = train(model, place, "native", steps=5, init=init)
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6)
    for k in ref_p:
        np.testing.assert_allclose(got_p[k], ref_p[k], rtol=1e-4, atol=1e-5, err_msg=k)
    assert exe._native.host_fallbacks() == {}, exe._native.host_fallbacks()


def test_native_engine_links_the_kernel_library():
    """The native executor's device kernels are the kernel library's: both .so files
    are mapped once a device engine ran."""
    place = fluid.CUDAPlace(0)
    train("lenet", place, "native", steps=1)
    maps = open("/proc/self/maps").read()
    assert "libpaddle_amd_native.so" in maps and "libpaddle_amd_kernels.so" in maps
    lib = os.path.join(os.path.dirname(fluid.__file__), "..", "lib", "libpaddle_amd_native.so")
    assert os.path.exists(lib)


def test_native_sequence_ops_device_kernels():
    """sequence_pool / sequence_softmax (+ grads) as device kernels of the native
    executor (ops_gpu.hip on pa_seq_pool / pa_seq_softmax_*): no host fallback, same
    trajectory as the Python executor."""
    from test_native_engine_cpu import seq_ops_trajectories

    ref, got, fb = seq_ops_trajectories(fluid.CUDAPlace(0))
    assert not any(k.startswith("sequence_") for k in fb), fb
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5)
