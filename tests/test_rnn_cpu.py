"""CPU checks of the LSTM reference recurrence used as the numerics oracle of the
persistent kernel (tests/test_rnn_gpu.py)."""
import torch

from paddle_amd.ops import rnn


def test_lstm_ref_matches_torch_lstm():
    torch.manual_seed(0)
    T, B, I, H = 6, 3, 5, 8
    m = torch.nn.LSTM(I, H)
    x = torch.randn(T, B, I)
    out, (h, c) = m(x)
    w_ih, w_hh = m.weight_ih_l0.t(), m.weight_hh_l0.t()
    b = m.bias_ih_l0 + m.bias_hh_l0
    hs, hl, cl = rnn.lstm(x, w_ih, w_hh, b)
    torch.testing.assert_close(hs, out, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(hl, h[0], rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(cl, c[0], rtol=1e-5, atol=1e-6)


def test_lstm_ref_lengths_freeze_state():
    torch.manual_seed(1)
    T, B, I, H = 6, 3, 4, 5
    x = torch.randn(T, B, I)
    w_ih, w_hh, b = torch.randn(I, 4 * H), torch.randn(H, 4 * H), torch.randn(4 * H)
    lens = torch.tensor([6, 2, 4])
    hs, hl, _ = rnn.lstm(x, w_ih, w_hh, b, lens=lens)
    for j in range(B):
        solo, hj, _ = rnn.lstm(x[: lens[j], j:j + 1], w_ih, w_hh, b)
        torch.testing.assert_close(hl[j], hj[0])
        torch.testing.assert_close(hs[: lens[j], j], solo[:, 0])
        assert torch.equal(hs[lens[j]:, j], hj.expand(T - lens[j], H))


def test_reverse_padded_cpu():
    x = torch.arange(12.0).view(4, 3)
    lens = torch.tensor([4, 1, 3])
    r = rnn.reverse_padded(x, lens)
    assert r[:, 0].tolist() == [9.0, 6.0, 3.0, 0.0]
    assert r[:, 1].tolist() == x[:, 1].tolist()
    assert r[:3, 2].tolist() == [8.0, 5.0, 2.0] and r[3, 2] == 11.0


def test_attention_decoder_ref_grad_shapes():
    torch.manual_seed(0)
    B, Ts, E, A, H, Tt = 2, 5, 8, 6, 4, 3
    enc = torch.randn(B, Ts, E, requires_grad=True)
    ep = torch.randn(B, Ts, A, requires_grad=True)
    lens = torch.tensor([5, 2])
    Y = torch.randn(Tt, B, 4 * H, requires_grad=True)
    h0, c0 = torch.zeros(B, H), torch.zeros(B, H)
    Wsp, w, Wg = torch.randn(H, A), torch.randn(A), torch.randn(E + H, 4 * H)
    out = rnn.attention_lstm_decoder(enc, ep, lens, Y, h0, c0, Wsp, w, Wg)
    assert out.shape == (Tt, B, H)
    out.sum().backward()
    # masked source positions get no attention and no gradient
    assert enc.grad[1, 2:].abs().sum() == 0 and ep.grad[1, 2:].abs().sum() == 0
