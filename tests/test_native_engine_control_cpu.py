"""Step scopes, tensor arrays, rank tables and SelectedRows on the C++ executor
(VERDICT r4 item 5): DynamicRNN training (while + while_grad over kept step scopes)
and word2vec with a shared is_sparse embedding (SelectedRows W@GRAD, sparse SGD /
Adam) run under ``engine="native"`` with NO Python-kernel fallback and follow the
Python engine's trajectory to 1e-5.  Reference: operators/while_op.cc:36-131,
framework/executor.cc:56-88, lookup_table_op.cc (SelectedRows grad), sgd_op.h,
adam_op.h."""
import numpy as np
import pytest

import paddle_amd.fluid as fluid

from native_control_cases import CASES, run


@pytest.mark.parametrize("case", sorted(CASES))
def test_control_program_native_matches_python(case):
    build, feeds = CASES[case]
    fd = feeds()
    place = fluid.CPUPlace()
    ref, init, _ = run(build, fd, "python", place)
    got, _, exe = run(build, fd, "native", place, init=init)
    assert exe._native is not None and exe._native.binding in ("pybind", "ctypes")
    for r, g in zip(ref, got):
        for a, b in zip(r, g):
            np.testing.assert_allclose(b, a, rtol=1e-5, atol=1e-6)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks


def test_drnn_native_trains():
    build, feeds = CASES["drnn_train"]
    got, _, exe = run(build, feeds(20), "native", fluid.CPUPlace())
    ls = [float(np.asarray(g[0]).reshape(-1)[0]) for g in got]
    assert ls[-1] < 0.5 * ls[0], ls


def test_native_can_run_accepts_control_and_sparse_programs():
    from paddle_amd.fluid.native_engine import NativeEngine

    for case in ("drnn_train", "word2vec_sparse_adam"):
        main, startup = fluid.Program(), fluid.Program()
        with fluid.unique_name.guard(), fluid.program_guard(main, startup):
            CASES[case][0]()
        assert NativeEngine.can_run(main, fluid.CPUPlace()), case


def test_device_ops_program_native_matches_python():
    from native_control_cases import CASES_DEVICE_OPS

    build, feeds = CASES_DEVICE_OPS["device_ops"]
    fd = feeds()
    ref, init, _ = run(build, fd, "python", fluid.CPUPlace())
    got, _, exe = run(build, fd, "native", fluid.CPUPlace(), init=init)
    for r, g in zip(ref, got):
        for a, b in zip(r, g):
            np.testing.assert_allclose(np.asarray(b, dtype="float64"), np.asarray(a, dtype="float64"),
                                       rtol=1e-5, atol=1e-6)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks


def test_every_host_kernel_has_a_device_kernel():
    """on a HIP place no registered op may need the host-copy
    fallback for lack of a device kernel (metadata-only ops are place-agnostic)."""
    from paddle_amd import native

    host, dev = set(native.registered_ops(False)), set(native.registered_ops(True))
    agnostic = {"feed", "fetch", "reshape", "reshape2", "flatten", "flatten2", "squeeze", "squeeze2", "unsqueeze",
                "unsqueeze2", "delete_var", "reshape_grad", "reshape2_grad"}
    assert host - dev - agnostic == set()


def test_conditional_block_grad_matches_unconditional_program():
    """With the condition true the block's gradients equal those of the same layers
    outside any block; with it false every input gradient is zero."""
    import torch

    def plain():
        L = fluid.layers
        x = L.data(name="x", shape=[4], dtype="float32")
        x.stop_gradient = False
        h = L.fc(x, size=3, act="tanh", param_attr=fluid.ParamAttr(name="cw"), bias_attr=fluid.ParamAttr(name="cb"))
        loss = L.mean(L.elementwise_mul(h, h))
        pg = fluid.backward.append_backward(loss)
        return [loss, "x@GRAD"] + [g for _, g in pg]

    from native_control_cases import cond_block_feeds

    fd = cond_block_feeds()
    place = fluid.CPUPlace()
    on, init, _ = run(CASES["cond_block_true"][0], fd, "python", place)
    ref, _, _ = run(plain, fd, "python", place, init={k: v for k, v in init.items() if k in ("cw", "cb")})
    for a, b in zip(on[0], ref[0]):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)
    off, _, _ = run(CASES["cond_block_false"][0], fd, "python", place, init=init)
    assert float(np.asarray(off[0][0]).reshape(-1)[0]) == 0.0
    for g in off[0][1:]:
        assert not np.any(np.asarray(g)), g
    del torch
