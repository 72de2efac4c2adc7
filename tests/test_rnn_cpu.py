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
