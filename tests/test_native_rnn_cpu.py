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


def test_book_label_semantic_roles_native():
    """The book SRL model (db_lstm + linear_chain_crf + crf_decoding, SGD with
    exponential_decay) runs entirely on the C++ executor and follows the interpreter."""
    from native_rnn_cases import srl, srl_feeds

    fd = srl_feeds(4)
    place = fluid.CPUPlace()
    ref, init, _ = run(srl(), fd, "python", place)
    got, _, exe = run(srl(), fd, "native", place, init)
    for a, b in zip(ref, got):
        np.testing.assert_allclose(b[0], a[0], rtol=1e-5, atol=1e-6)
        np.testing.assert_array_equal(b[1], a[1])
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks


def test_book_machine_translation_train_and_beam_decode_native():
    """Book machine_translation: the training program (LSTM encoder, DynamicRNN
    decoder, Adagrad + L2) and the beam-search decoding program (While, topk,
    beam_search over tensor arrays, beam_search_decode) on the C++ executor."""
    from native_rnn_cases import mt_decode, mt_decode_feeds, mt_train, mt_train_feeds

    place = fluid.CPUPlace()
    fd = mt_train_feeds(4)
    ref, init, _ = run(mt_train, fd, "python", place)
    got, _, exe = run(mt_train, fd, "native", place, init)
    for a, b in zip(ref, got):
        np.testing.assert_allclose(b[0], a[0], rtol=1e-5, atol=1e-6)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks
    fd = mt_decode_feeds(2)
    ref, init, _ = run(mt_decode, fd, "python", place)
    got, _, exe = run(mt_decode, fd, "native", place, init)
    for a, b in zip(ref, got):
        np.testing.assert_array_equal(b[0], a[0])
        np.testing.assert_allclose(b[1], a[1], rtol=1e-5, atol=1e-6)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks


def test_sequence_row_map_ops_native():
    from native_rnn_cases import seq_ops_feeds, seq_ops_net

    fd = seq_ops_feeds(4)
    place = fluid.CPUPlace()
    ref, init, _ = run(seq_ops_net(), fd, "python", place)
    got, _, exe = run(seq_ops_net(), fd, "native", place, init)
    for a, b in zip(ref, got):
        np.testing.assert_allclose(b[0], a[0], rtol=1e-5, atol=1e-6)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks


def test_static_rnn_native():
    from native_rnn_cases import static_rnn, static_rnn_feeds

    fd = static_rnn_feeds(4)
    place = fluid.CPUPlace()
    ref, init, _ = run(static_rnn(), fd, "python", place)
    got, _, exe = run(static_rnn(), fd, "native", place, init)
    for a, b in zip(ref, got):
        np.testing.assert_allclose(b[0], a[0], rtol=1e-5, atol=1e-6)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks


def test_layout_ops_native():
    from native_rnn_cases import layout_feeds, layout_net

    fd = layout_feeds(4)
    place = fluid.CPUPlace()
    ref, init, _ = run(layout_net(), fd, "python", place)
    got, _, exe = run(layout_net(), fd, "native", place, init)
    for a, b in zip(ref, got):
        np.testing.assert_allclose(b[0], a[0], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(b[1], a[1], rtol=1e-5, atol=1e-6)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks


def test_rnn_unit_ops_native():
    """gru_unit / lstm_unit (+ grads) on the one-source host kernels of ops_rnn_unit.hip."""
    from native_rnn_cases import units_feeds, units_net

    fd = units_feeds(4)
    place = fluid.CPUPlace()
    ref, init, _ = run(units_net(), fd, "python", place)
    got, _, exe = run(units_net(), fd, "native", place, init)
    for a, b in zip(ref, got):
        np.testing.assert_allclose(b[0], a[0], rtol=1e-5, atol=1e-6)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks


def test_conv3d_pool3d_native():
    from native_rnn_cases import vol_feeds, vol_net

    fd = vol_feeds(4)
    place = fluid.CPUPlace()
    ref, init, _ = run(vol_net(), fd, "python", place)
    got, _, exe = run(vol_net(), fd, "native", place, init)
    for a, b in zip(ref, got):
        np.testing.assert_allclose(b[0], a[0], rtol=1e-5, atol=1e-6)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks


def test_structured_losses_native():
    """warpctc / nce / hierarchical_sigmoid / roi_pool (+grads) and edit_distance on
    ops_loss.hip's host kernels."""
    from native_rnn_cases import losses_feeds, losses_net

    fd = losses_feeds(4)
    place = fluid.CPUPlace()
    ref, init, _ = run(losses_net(), fd, "python", place)
    got, _, exe = run(losses_net(), fd, "native", place, init)
    for a, b in zip(ref, got):
        np.testing.assert_allclose(b[0], a[0], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(b[1], a[1], rtol=1e-6)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks


@pytest.mark.parametrize("reverse", [False, True])
def test_recurrent_op_native_matches_interpreter(reverse):
    """The `recurrent` op (the reference StaticRNN's) and its recurrent_grad run on the
    C++ executor over kept step scopes (core.cc RunRecurrent / RunRecurrentGrad): two
    inputs, two linked states, a trainable initial state, SGD; the loss trajectory and
    every gradient match the interpreter, and an independent torch unroll."""
    import torch

    from native_rnn_cases import recurrent_feeds, recurrent_net

    fd = recurrent_feeds(3)
    place = fluid.CPUPlace()
    ref, init, _ = run(recurrent_net(reverse), fd, "python", place)
    init0 = {k: v.copy() for k, v in init.items()}  # the runs train their scope's arrays in place
    got, _, exe = run(recurrent_net(reverse), fd, "native", place, init)
    init = init0
    for a, b in zip(ref, got):
        for x, y in zip(a, b):
            np.testing.assert_allclose(y, x, rtol=1e-5, atol=1e-6)
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks
    # step 0 against torch autograd
    W = torch.tensor(init["rw"], requires_grad=True)
    U = torch.tensor(init["ru"], requires_grad=True)
    H0 = torch.tensor(init["rh0"], requires_grad=True)
    X1 = torch.tensor(fd[0]["rx1"], requires_grad=True)
    X2 = torch.tensor(fd[0]["rx2"])
    h, c = H0, torch.full_like(H0, 0.5)
    ys, hs = [None] * 5, [None] * 5
    for t in (range(4, -1, -1) if reverse else range(5)):
        h = torch.tanh(X1[t] @ W + h @ U + X2[t])
        c = c * h
        ys[t], hs[t] = c + h, h
    Y, Hs = torch.stack(ys), torch.stack(hs)
    loss = (Y * Y).mean() + Hs.mean()
    loss.backward()
    np.testing.assert_allclose(got[0][0], loss.detach().numpy().reshape(got[0][0].shape), rtol=1e-5)
    for arr, ref_t in zip(got[0][2:], (X1, H0, W, U)):
        np.testing.assert_allclose(arr, ref_t.grad.numpy(), rtol=1e-4, atol=1e-6)
