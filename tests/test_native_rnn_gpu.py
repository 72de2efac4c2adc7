"""The LoD lstm / gru programs of test_native_rnn_cpu.py on a HIP place: the device
kernels (csrc/native/ops_rnn_gpu.hip -- one pa_sgemm per time step plus a fused cell
kernel) run every recurrent op, forward and grad, with no Python-kernel fallback and
no host round trip, following the interpreter on the same device to 2e-4."""
import numpy as np
import pytest

import paddle_amd.fluid as fluid

from native_control_cases import run
from native_rnn_cases import CASES, feeds

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", sorted(CASES))
def test_native_rnn_matches_interpreter_gpu(case):
    build, kw = CASES[case]
    fd = feeds(4, **kw)
    place = fluid.CUDAPlace(0)
    ref, init, _ = run(build, fd, "python", place)
    got, _, exe = run(build, fd, "native", place, init)
    for a, b in zip(ref, got):
        np.testing.assert_allclose(b[0], a[0], rtol=2e-4, atol=2e-5)
    eng = exe._native
    assert not eng.py_fallbacks, eng.py_fallbacks
    assert not eng.host_fallbacks(), eng.host_fallbacks()


def test_book_label_semantic_roles_native_gpu():
    """Book SRL (db_lstm + linear_chain_crf + crf_decoding) on the device kernels:
    no Python fallback, no host round trip; decoded paths equal the interpreter's."""
    from native_rnn_cases import srl, srl_feeds

    fd = srl_feeds(4)
    place = fluid.CUDAPlace(0)
    ref, init, _ = run(srl(), fd, "python", place)
    got, _, exe = run(srl(), fd, "native", place, init)
    for a, b in zip(ref, got):
        np.testing.assert_allclose(b[0], a[0], rtol=2e-4, atol=2e-5)
        np.testing.assert_array_equal(b[1], a[1])
    eng = exe._native
    assert not eng.py_fallbacks, eng.py_fallbacks
    assert not eng.host_fallbacks(), eng.host_fallbacks()


def test_book_machine_translation_native_gpu():
    """Book machine_translation train + beam decode on a HIP place: the recurrent,
    optimizer (adagrad) and decoding ops run natively (beam_search /
    beam_search_decode are place-agnostic kernels over their few-KB inputs, as the
    reference registers them CPU-only)."""
    from native_rnn_cases import mt_decode, mt_decode_feeds, mt_train, mt_train_feeds

    place = fluid.CUDAPlace(0)
    fd = mt_train_feeds(4)
    ref, init, _ = run(mt_train, fd, "python", place)
    got, _, exe = run(mt_train, fd, "native", place, init)
    for a, b in zip(ref, got):
        np.testing.assert_allclose(b[0], a[0], rtol=2e-4, atol=2e-5)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks
    assert not exe._native.host_fallbacks(), exe._native.host_fallbacks()
    fd = mt_decode_feeds(2)
    ref, init, _ = run(mt_decode, fd, "python", place)
    got, _, exe = run(mt_decode, fd, "native", place, init)
    for a, b in zip(ref, got):
        np.testing.assert_array_equal(b[0], a[0])
        np.testing.assert_allclose(b[1], a[1], rtol=2e-4, atol=2e-5)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks
    assert not exe._native.host_fallbacks(), exe._native.host_fallbacks()


def test_sequence_row_map_ops_native_gpu():
    """sequence_conv / pad / unpad / slice / erase / mask / enumerate (ops_seq.cc:
    row maps on the host, rows moved by the device gather / scatter kernels)."""
    from native_rnn_cases import seq_ops_feeds, seq_ops_net

    fd = seq_ops_feeds(4)
    place = fluid.CUDAPlace(0)
    ref, init, _ = run(seq_ops_net(), fd, "python", place)
    got, _, exe = run(seq_ops_net(), fd, "native", place, init)
    for a, b in zip(ref, got):
        np.testing.assert_allclose(b[0], a[0], rtol=2e-4, atol=2e-5)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks
    assert not exe._native.host_fallbacks(), exe._native.host_fallbacks()


@pytest.mark.parametrize("case", ["static_rnn", "layout", "units", "vol", "losses", "recurrent", "recurrent_rev"])
def test_layout_ops_native_gpu(case):
    """The unrolled StaticRNN (slice / squeeze / stack per step) and the layout-op
    chain on a HIP place: ops_tensor.hip's strided-box kernel moves every tensor."""
    import native_rnn_cases as C

    build, feeds_fn = {"static_rnn": (C.static_rnn, C.static_rnn_feeds),
                       "layout": (C.layout_net, C.layout_feeds),
                       "units": (C.units_net, C.units_feeds),
                       "vol": (C.vol_net, C.vol_feeds),
                       "losses": (C.losses_net, C.losses_feeds),
                       "recurrent": (lambda: C.recurrent_net(False), C.recurrent_feeds),
                       "recurrent_rev": (lambda: C.recurrent_net(True), C.recurrent_feeds)}[case]
    fd = feeds_fn(4)
    place = fluid.CUDAPlace(0)
    ref, init, _ = run(build(), fd, "python", place)
    got, _, exe = run(build(), fd, "native", place, init)
    for a, b in zip(ref, got):
        for x, y in zip(a, b):
            np.testing.assert_allclose(y, x, rtol=2e-4, atol=2e-5)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks
    assert not exe._native.host_fallbacks(), exe._native.host_fallbacks()
