"""The framework's DyGraph eager engine (paddle_amd/autograd/engine.py + rules.py).

* Every backward rule is checked against an oracle: torch autograd on raw fp64
  tensors of the same op (reference semantics; the engine itself never calls it).
* BASELINE config 1 (MNIST LeNet DyGraph on CPUPlace) and a ResNet-tiny bf16 step
  train with ``torch.autograd.backward`` / ``torch.autograd.grad`` patched to raise,
  and without any op taking the engine's torch-autograd fallback.
* Engine semantics: paddle.grad (leaf and intermediate), no_grad, retain_graph,
  gradient hooks, in-place / setitem, stop_gradient, grad-ready hooks.
Reference behaviour: python/paddle/fluid/backward.py (gradient accumulation of
repeated uses, _addup_repetitive_outputs_:135), Paddle 2.x ``paddle.grad``.
"""
import contextlib

import numpy as np
import pytest
import torch
import torch.nn.functional as TF

import paddle
import paddle.nn as nn
import paddle.nn.functional as F
from paddle_amd.autograd import engine


@contextlib.contextmanager
def no_torch_autograd():
    """torch.autograd entry points raise while the block runs."""
    saved = (torch.autograd.backward, torch.autograd.grad, torch.Tensor.backward)

    def boom(*a, **k):
        raise AssertionError("torch.autograd was called")

    torch.autograd.backward = boom
    torch.autograd.grad = boom
    torch.Tensor.backward = boom
    before = dict(engine.FALLBACK_OPS)
    try:
        yield
    finally:
        torch.autograd.backward, torch.autograd.grad, torch.Tensor.backward = saved
    assert engine.FALLBACK_OPS == before, f"ops took the torch-autograd fallback: {engine.FALLBACK_OPS}"


def _pt(x, sg=False):
    return paddle.to_tensor(x, stop_gradient=sg)


R = np.random.RandomState(0)
A34 = R.randn(3, 4)
B34 = R.randn(3, 4)
B14 = R.randn(1, 4)
P34 = R.rand(3, 4) + 0.5
M45 = R.randn(4, 5)
X4 = R.randn(2, 3, 6, 6)
Y34 = (R.rand(3, 4) > 0.5).astype(np.float64)
W4 = R.randn(4, 3, 3, 3)

# (name, fn(*tensors), inputs): fn is applied to framework Tensors (engine) and to raw
# fp64 torch tensors (oracle); gradients of a random projection of the output match
CASES = [
    ("add_bcast", lambda a, b: a + b, [A34, B14]),
    ("radd", lambda a: 2.0 + a, [A34]),
    ("sub", lambda a, b: a - b, [A34, B34]),
    ("rsub", lambda a: 1.0 - a, [A34]),
    ("mul", lambda a, b: a * b, [A34, B14]),
    ("div", lambda a, b: a / b, [A34, P34]),
    ("rdiv", lambda a: 2.0 / a, [P34]),
    ("pow", lambda a: a ** 3, [A34]),
    ("pow_t", lambda a, b: a ** b, [P34, B34]),
    ("rpow", lambda a: 2.0 ** a, [A34]),
    ("neg", lambda a: -a, [A34]),
    ("exp", torch.exp, [A34]), ("log", torch.log, [P34]), ("sqrt", torch.sqrt, [P34]),
    ("rsqrt", torch.rsqrt, [P34]), ("abs", torch.abs, [A34]), ("sin", torch.sin, [A34]),
    ("cos", torch.cos, [A34]), ("tanh", torch.tanh, [A34]), ("sigmoid", torch.sigmoid, [A34]),
    ("relu", TF.relu, [A34]), ("relu6", lambda a: TF.relu6(a * 4), [A34]), ("leaky", TF.leaky_relu, [A34]),
    ("elu", TF.elu, [A34]), ("gelu", TF.gelu, [A34]), ("gelu_tanh", lambda a: TF.gelu(a, approximate="tanh"), [A34]),
    ("silu", TF.silu, [A34]), ("softplus", TF.softplus, [A34]), ("hardswish", lambda a: TF.hardswish(a * 3), [A34]),
    ("mish", TF.mish, [A34]), ("erf", torch.erf, [A34]), ("square", torch.square, [A34]),
    ("clamp", lambda a: a.clamp(-0.5, 0.5), [A34]), ("maximum", torch.maximum, [A34, B34]),
    ("where", lambda a, b: torch.where(a > 0, a, b), [A34, B34]),
    ("matmul", lambda a, b: a @ b, [A34, M45]), ("matmul_vec", lambda a, b: a @ b, [A34, R.randn(4)]),
    ("bmm", torch.bmm, [R.randn(2, 3, 4), R.randn(2, 4, 5)]),
    ("linear", lambda x, w, b: TF.linear(x, w, b), [A34, R.randn(5, 4), R.randn(5)]),
    ("addmm", lambda c, a, b: torch.addmm(c, a, b, beta=0.5, alpha=2.0), [R.randn(3, 5), A34, M45]),
    ("sum", lambda a: a.sum(), [A34]), ("sum_dim", lambda a: a.sum(1, keepdim=True), [A34]),
    ("mean", lambda a: a.mean(0), [A34]), ("max_dim", lambda a: a.max(1)[0], [A34]),
    ("max_all", lambda a: a.max(), [A34]), ("amax", lambda a: a.amax(1), [A34]),
    ("logsumexp", lambda a: torch.logsumexp(a, 1), [A34]), ("var", lambda a: a.var(1), [A34]),
    ("std", lambda a: a.std(0), [A34]), ("norm", lambda a: a.norm(), [A34]), ("cumsum", lambda a: a.cumsum(1), [A34]),
    ("reshape", lambda a: a.reshape(4, 3) * torch.arange(12.0, dtype=a.dtype).reshape(4, 3), [A34]),
    ("transpose", lambda a: a.t() @ a, [A34]), ("permute", lambda a: a.permute(2, 0, 1), [R.randn(2, 3, 4)]),
    ("expand", lambda a: a.expand(3, 4) * 2, [B14]), ("repeat", lambda a: a.repeat(2, 3), [A34]),
    ("getitem", lambda a: a[1:, ::2] * 3, [A34]), ("getitem_adv", lambda a: a[torch.tensor([0, 2, 0])], [A34]),
    ("cat", lambda a, b: torch.cat([a, b], 0), [A34, B34]), ("stack", lambda a, b: torch.stack([a, b], 1), [A34, B34]),
    ("split", lambda a: torch.split(a, [1, 3], 1)[1] * 2, [A34]), ("chunk", lambda a: a.chunk(2, 1)[0], [A34]),
    ("unbind", lambda a: a.unbind(0)[2], [A34]), ("gather", lambda a: a.gather(1, torch.tensor([[0, 1], [2, 3],
                                                                                                   [1, 1]])), [A34]),
    ("index_select", lambda a: a.index_select(1, torch.tensor([3, 0, 3])), [A34]),
    ("masked_fill", lambda a: a.masked_fill(a > 0.5, 0.0), [A34]), ("flip", lambda a: a.flip(1), [A34]),
    ("squeeze", lambda a: a.unsqueeze(0).squeeze(0), [A34]), ("flatten", lambda a: a.flatten(), [R.randn(2, 3, 4)]),
    ("pad", lambda a: TF.pad(a, (1, 2)), [A34]), ("tril", torch.tril, [R.randn(4, 4)]),
    ("softmax", lambda a: TF.softmax(a, -1), [A34]), ("log_softmax", lambda a: TF.log_softmax(a, 1), [A34]),
    ("conv2d", lambda x, w: TF.conv2d(x, w, stride=1, padding=1), [X4, W4]),
    ("conv2d_bias_stride", lambda x, w, b: TF.conv2d(x, w, b, 2, 1), [X4, W4, R.randn(4)]),
    ("conv_t2d", lambda x, w: TF.conv_transpose2d(x, w, stride=2), [X4, R.randn(3, 2, 3, 3)]),
    ("maxpool", lambda x: TF.max_pool2d(x, 2, 2), [X4]), ("avgpool", lambda x: TF.avg_pool2d(x, 3, 2, 1), [X4]),
    ("aap", lambda x: TF.adaptive_avg_pool2d(x, 1), [X4]),
    ("bn_train", lambda x, w, b: TF.batch_norm(x, torch.zeros(3, dtype=x.dtype), torch.ones(3, dtype=x.dtype), w, b,
                                               True), [X4, R.rand(3) + 0.5, R.randn(3)]),
    ("ln", lambda x, w, b: TF.layer_norm(x, (6,), w, b), [X4, R.rand(6) + 0.5, R.randn(6)]),
    ("gn", lambda x, w, b: TF.group_norm(x, 3, w, b), [X4, R.rand(3) + 0.5, R.randn(3)]),
    ("embedding", lambda w: TF.embedding(torch.tensor([[1, 3], [3, 0]]), w), [R.randn(5, 4)]),
    ("ce", lambda x: TF.cross_entropy(x, torch.tensor([1, 0, 3])), [A34]),
    ("ce_ignore_w", lambda x: TF.cross_entropy(x, torch.tensor([1, -100, 3]), torch.tensor([0.5, 1.0, 2.0, 1.5],
                                                                                           dtype=x.dtype)), [A34]),
    ("ce_nd_sum", lambda x: TF.cross_entropy(x, torch.tensor([[1, 0], [2, 2]]), reduction="sum"),
     [R.randn(2, 3, 2)]),
    ("nll", lambda x: TF.nll_loss(TF.log_softmax(x, 1), torch.tensor([2, 0, 1])), [A34]),
    ("mse", lambda a, b: TF.mse_loss(a, b), [A34, B34]), ("l1", lambda a, b: TF.l1_loss(a, b, reduction="sum"),
                                                          [A34, B34]),
    ("smooth_l1", lambda a, b: TF.smooth_l1_loss(a, b), [A34, B34 * 3]),
    ("bce_logits", lambda a: TF.binary_cross_entropy_with_logits(a, torch.tensor(Y34, dtype=a.dtype)), [A34]),
    ("bce", lambda a: TF.binary_cross_entropy(torch.sigmoid(a), torch.full_like(a, 0.3)), [A34]),
    ("cos_sim", lambda a, b: TF.cosine_similarity(a, b), [A34, B34]),
    ("normalize", lambda a: TF.normalize(a, dim=1), [A34]),
    ("to_dtype", lambda a: a.float().double() * 2, [A34]),
    ("sum_reuse", lambda a: (a * a).sum() + a.sum(), [A34]),
]


@pytest.mark.parametrize("name,fn,inputs", CASES, ids=[c[0] for c in CASES])
def test_rule_matches_oracle(name, fn, inputs):
    raw = [torch.tensor(x, dtype=torch.float64, requires_grad=True) for x in inputs]
    out_ref = fn(*raw)
    proj = torch.tensor(np.random.RandomState(1).randn(*out_ref.shape)) if out_ref.dim() else torch.tensor(1.3,
                                                                                                         dtype=torch.float64)
    (out_ref * proj).sum().backward()
    ours = [_pt(torch.tensor(x, dtype=torch.float64)) for x in inputs]
    before = dict(engine.FALLBACK_OPS)
    with no_torch_autograd():
        out = fn(*ours)
        assert isinstance(out, paddle.Tensor)
        (out * proj).sum().backward()
    assert engine.FALLBACK_OPS == before
    np.testing.assert_allclose(out.detach().numpy(), out_ref.detach().numpy(), rtol=1e-10, atol=1e-10)
    for o, r in zip(ours, raw):
        assert o.grad is not None, name
        np.testing.assert_allclose(o.grad.numpy(), r.grad.numpy(), rtol=1e-7, atol=1e-9, err_msg=name)


def _mnist(n=384, bs=64):
    ds = paddle.vision.datasets.MNIST(mode="train", num_samples=n)
    return paddle.io.DataLoader(ds, batch_size=bs, shuffle=True)


def test_lenet_dygraph_cpu_trains_without_torch_autograd():
    """BASELINE config 1 on the framework engine only."""
    paddle.seed(3)
    paddle.set_device("cpu")
    model = paddle.vision.models.LeNet()
    for p in model.parameters():
        assert isinstance(p, paddle.Tensor) and not p.stop_gradient
    opt = paddle.optimizer.Adam(learning_rate=2e-3, parameters=model.parameters())
    first = last = None
    with no_torch_autograd():
        for _ in range(2):
            for img, label in _mnist():
                loss = F.cross_entropy(model(img), label)
                assert loss.grad_node is not None
                loss.backward()
                opt.step()
                opt.clear_grad()
                first = float(loss) if first is None else first
                last = float(loss)
    assert last < first * 0.6, (first, last)


def test_resnet_tiny_bf16_step_without_torch_autograd():
    paddle.seed(0)
    paddle.set_device("cpu")
    model = paddle.vision.models.resnet18(num_classes=10)
    model.to(dtype=torch.bfloat16)
    opt = paddle.optimizer.Momentum(learning_rate=0.05, momentum=0.9, parameters=model.parameters())
    x = paddle.randn([4, 3, 32, 32]).astype("bfloat16")
    y = paddle.to_tensor(np.array([1, 3, 5, 7]))
    losses = []
    with no_torch_autograd():
        for _ in range(4):
            loss = F.cross_entropy(model(x).astype("float32"), y)
            loss.backward()
            for p in model.parameters():
                assert p.grad is not None and p.grad.dtype == torch.bfloat16
            opt.step()
            opt.clear_grad()
            losses.append(float(loss))
    assert losses[-1] < losses[0], losses


def test_paddle_grad_leaf_and_intermediate():
    x = _pt(np.array([1.0, 2.0, 3.0]))
    with no_torch_autograd():
        y = x * x
        z = (y * 3).sum()
        gx, gy = paddle.grad([z], [x, y], retain_graph=True)
        np.testing.assert_allclose(gx.numpy(), 6 * x.detach().numpy())
        np.testing.assert_allclose(gy.numpy(), [3.0, 3.0, 3.0])
        assert x.grad is None  # paddle.grad does not touch .grad
        z.backward()
    np.testing.assert_allclose(x.grad.numpy(), 6 * x.detach().numpy())


def test_accumulation_no_grad_retain_and_hooks():
    x = _pt(np.ones(3))
    seen = []
    x.register_hook(lambda g: seen.append(g.numpy().copy()))
    with no_torch_autograd():
        (x * 2).sum().backward()
        (x * 3).sum().backward()  # accumulates
        np.testing.assert_allclose(x.grad.numpy(), [5.0] * 3)
        with paddle.no_grad():
            y = x * 4
        assert y.stop_gradient and y.grad_node is None
        z = (x * x).sum()
        z.backward(retain_graph=True)
        z.backward()
    np.testing.assert_allclose(x.grad.numpy(), [9.0] * 3)
    assert len(seen) == 4
    w = (x * 1).sum()
    w.backward()
    with pytest.raises(RuntimeError):
        w.backward()  # graph freed


def test_inplace_and_setitem():
    x = _pt(np.arange(4.0))
    with pytest.raises(RuntimeError):
        x.add_(1.0)  # leaf that requires grad
    with no_torch_autograd():
        y = x * 1.0
        y.mul_(3.0)
        y[1] = 0.0
        y.sum().backward()
    np.testing.assert_allclose(x.grad.numpy(), [3.0, 0.0, 3.0, 3.0])
    a = _pt(np.ones(3))
    b = paddle.zeros([3])
    with no_torch_autograd():
        b[0:2] = a[0:2] * 5  # untracked target takes the source's gradient
        b.sum().backward()
    np.testing.assert_allclose(a.grad.numpy(), [5.0, 5.0, 0.0])


def test_stop_gradient_and_grad_ready_hooks():
    p = nn.Linear(3, 2).weight
    fired = []
    p._pa_grad_ready_hooks = [lambda t: fired.append(t.grad.clone())]
    x = paddle.randn([4, 3])
    assert x.stop_gradient
    with no_torch_autograd():
        loss = (x @ p).sum() + (x @ p * 2).sum()  # two uses: hook fires once, after both
        loss.backward()
    assert len(fired) == 1 and torch.allclose(fired[0], p.grad)
    p.stop_gradient = True
    assert not p.requires_grad
    y = x @ p
    assert y.stop_gradient


def test_framework_tensor_is_returned_by_paddle_api():
    for t in (paddle.zeros([2]), paddle.ones([2, 2]), paddle.randn([3]), paddle.arange(4), paddle.to_tensor([1.0]),
              paddle.concat([paddle.ones([1]), paddle.ones([1])]), paddle.matmul(paddle.ones([2, 2]),
                                                                                paddle.ones([2, 2]))):
        assert isinstance(t, paddle.Tensor), type(t)
    assert paddle.to_tensor([1.0, 2.0]).astype("float64").dtype == torch.float64
    assert paddle.to_tensor([1.0]).place == "cpu"


def test_fluid_lenet_trains_without_torch_autograd():
    """Fluid static-graph LeNet: the grad ops' kernels differentiate the forward
    kernels on the eager engine (framework/registry.py auto_grad_kernel), never on
    torch autograd."""
    import paddle_amd.fluid as fluid

    main, startup = fluid.Program(), fluid.Program()
    main.random_seed = startup.random_seed = 7
    with fluid.program_guard(main, startup):
        img = fluid.layers.data(name="img", shape=[1, 28, 28], dtype="float32")
        lab = fluid.layers.data(name="lab", shape=[1], dtype="int64")
        c1 = fluid.nets.simple_img_conv_pool(img, num_filters=8, filter_size=5, pool_size=2, pool_stride=2,
                                             act="relu")
        c2 = fluid.nets.simple_img_conv_pool(c1, num_filters=16, filter_size=5, pool_size=2, pool_stride=2,
                                             act="relu")
        pred = fluid.layers.fc(c2, size=10, act="softmax")
        loss = fluid.layers.mean(fluid.layers.cross_entropy(pred, lab))
        fluid.optimizer.Adam(learning_rate=6e-3).minimize(loss)
    ds = paddle.vision.datasets.MNIST(mode="train", num_samples=256)
    xs = np.stack([np.asarray(ds[i][0], dtype=np.float32).reshape(1, 28, 28) for i in range(256)])
    ys = np.array([int(np.asarray(ds[i][1]).reshape(-1)[0]) for i in range(256)], dtype=np.int64).reshape(-1, 1)
    exe = fluid.Executor(fluid.CPUPlace())
    scope = fluid.core.Scope()
    losses = []
    with fluid.executor.scope_guard(scope), no_torch_autograd():
        exe.run(startup)
        for ep in range(5):
            for b in range(0, 256, 64):
                out, = exe.run(main, feed={"img": xs[b:b + 64], "lab": ys[b:b + 64]}, fetch_list=[loss])
                losses.append(float(np.asarray(out).reshape(-1)[0]))
    assert losses[-1] < losses[0] * 0.7, losses
