"""The framework tape (autograd/tape.py): forward with torch autograd off, reverse
pass through hand-written Function backwards, activation grads by tag, parameter
grads + grad-ready hooks after the last use -- checked against torch autograd on
the same Functions (CPU)."""
import torch

from paddle_amd.autograd import tape


class _Lin(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return x @ w

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        return (g @ w.t() if ctx.needs_input_grad[0] else None), (x.t() @ g if ctx.needs_input_grad[1] else None)


class _Tanh2(torch.autograd.Function):
    """two outputs: (tanh(x), x * 2)"""

    @staticmethod
    def forward(ctx, x):
        y = torch.tanh(x)
        ctx.save_for_backward(y)
        return y, x * 2

    @staticmethod
    def backward(ctx, g1, g2):
        (y,) = ctx.saved_tensors
        out = 0
        if g1 is not None:
            out = out + g1 * (1 - y * y)
        if g2 is not None:
            out = out + 2 * g2
        return out


class _Mean(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.n = x.numel()
        ctx.shape = x.shape
        return x.mean()

    @staticmethod
    def backward(ctx, g):
        return g.expand(ctx.shape) / ctx.n


class _Add(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        return a + b

    @staticmethod
    def backward(ctx, g):
        return g, g


def _model(x, w1, w2):
    h = tape.apply(_Lin, x, w1)
    a, b = tape.apply(_Tanh2, h)
    y = tape.apply(_Lin, a, w2)
    z = tape.apply(_Lin, b, w2)          # w2 used twice: hooks fire once, after both
    return tape.apply(_Mean, tape.apply(_Lin, tape.apply(_Add, y, z), torch.ones(4, 1)))


def test_tape_matches_torch_autograd_and_fires_hooks_after_last_use():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(5, 3, generator=g)
    w1 = torch.randn(3, 4, generator=g, requires_grad=True)
    w2 = torch.randn(4, 4, generator=g, requires_grad=True)
    ref = _model(x, w1, w2)
    ref.backward()
    r1, r2 = w1.grad.clone(), w2.grad.clone()
    w1.grad = w2.grad = None
    fired = []
    for w in (w1, w2):
        w._pa_grad_ready_hooks = [lambda p: fired.append((p, p.grad.clone()))]
    with tape.recording() as t:
        assert not torch.is_grad_enabled()
        loss = _model(x, w1, w2)
        assert loss.grad_fn is None
    t.backward(loss)
    assert torch.allclose(loss, ref.detach())
    assert torch.allclose(w1.grad, r1) and torch.allclose(w2.grad, r2)
    # each hook once, with the complete gradient (w2's after both of its uses)
    assert [id(p) for p, _ in fired].count(id(w2)) == 1 and [id(p) for p, _ in fired].count(id(w1)) == 1
    assert torch.allclose(dict((id(p), gr) for p, gr in fired)[id(w2)], r2)
    assert not t.entries
