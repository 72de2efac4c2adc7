"""Optimizer.clear_grad(set_to_zero=True) zeroes every gradient with one fill per
(device, dtype): the gradients become views of a flat buffer on the first call and
stay there through the backward's in-place accumulation (no
per-parameter zero_ / full per step).  Training must be unchanged."""
import numpy as np
import torch

import paddle_amd as paddle


def _train(flat, steps=4):
    paddle.seed(3)
    net = paddle.nn.Sequential(paddle.nn.Linear(6, 5), paddle.nn.ReLU(), paddle.nn.Linear(5, 3))
    opt = paddle.optimizer.Momentum(learning_rate=0.1, momentum=0.9, parameters=net.parameters())
    if not flat:
        opt._flat_grad_zero = lambda: False
    rs = np.random.RandomState(0)
    losses = []
    for _ in range(steps):
        x = paddle.to_tensor(rs.randn(8, 6).astype("float32"))
        loss = (net(x) ** 2).mean()
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss))
    return losses, net, opt


def test_flat_grad_matches_per_tensor_clear():
    a, _, _ = _train(True)
    b, _, _ = _train(False)
    np.testing.assert_allclose(a, b, rtol=1e-6)


def test_grads_are_views_of_one_zeroed_buffer():
    _, net, opt = _train(True, steps=2)
    flat = opt._pa_flat_grads
    assert len(flat[2]) == 1
    buf = flat[2][0]
    lo, hi = buf.data_ptr(), buf.data_ptr() + buf.numel() * buf.element_size()
    for p in net.parameters():
        assert lo <= p.grad.data_ptr() < hi
        assert not torch.any(p.grad)
    # a user-rebound gradient is cleared by the per-tensor path, then re-homed
    p0 = list(net.parameters())[0]
    p0.grad = torch.ones_like(p0.grad)
    opt.clear_grad()
    assert not torch.any(p0.grad)
    opt.clear_grad()
    assert lo <= p0.grad.data_ptr() < hi or opt._pa_flat_grads[2][0].data_ptr() != lo
