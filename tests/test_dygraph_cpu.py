"""paddle.* 2.x DyGraph API on CPU: BASELINE config "MNIST LeNet DyGraph on
CPUPlace", .pdparams/.pdopt checkpoint round trip, optimizer and LR-schedule
numerics against closed-form references, layers, DataLoader, hapi.Model."""
import math
import os
import pickle

import numpy as np
import pytest
import torch

import paddle
import paddle.nn as nn
import paddle.nn.functional as F


def _mnist_loader(n=512, bs=64, shuffle=True, workers=0):
    ds = paddle.vision.datasets.MNIST(mode="train", num_samples=n)
    return paddle.io.DataLoader(ds, batch_size=bs, shuffle=shuffle, num_workers=workers)


def test_mnist_lenet_dygraph_cpu_converges():
    paddle.seed(1)
    paddle.set_device("cpu")
    model = paddle.vision.models.LeNet()
    opt = paddle.optimizer.Adam(learning_rate=1e-3, parameters=model.parameters())
    loss_fn = nn.CrossEntropyLoss()
    acc = paddle.metric.Accuracy()
    first = last = None
    for epoch in range(3):
        for img, label in _mnist_loader():
            out = model(img)
            loss = loss_fn(out, label)
            loss.backward()
            opt.step()
            opt.clear_grad()
            first = float(loss) if first is None else first
            last = float(loss)
            acc.update(acc.compute(out, label))
    assert last < first * 0.5
    assert acc.accumulate() > 0.5


def _train(model, opt, batches):
    for x, y in batches:
        loss = F.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        opt.clear_grad()
    return model


def test_pdparams_pdopt_roundtrip_resumes_exactly(tmp_path):
    paddle.set_device("cpu")
    batches = list(_mnist_loader(n=256, shuffle=False))
    sched = lambda: paddle.optimizer.lr.StepDecay(1e-3, step_size=2, gamma=0.5)  # noqa: E731

    paddle.seed(3)
    a = paddle.vision.models.LeNet()
    oa = paddle.optimizer.AdamW(learning_rate=sched(), parameters=a.parameters(), weight_decay=0.01)
    _train(a, oa, batches[:2])
    paddle.save(a.state_dict(), str(tmp_path / "m.pdparams"))
    paddle.save(oa.state_dict(), str(tmp_path / "m.pdopt"))
    _train(a, oa, batches[2:])

    paddle.seed(99)
    b = paddle.vision.models.LeNet()
    ob = paddle.optimizer.AdamW(learning_rate=sched(), parameters=b.parameters(), weight_decay=0.01)
    b.set_state_dict(paddle.load(str(tmp_path / "m.pdparams")))
    ob.set_state_dict(paddle.load(str(tmp_path / "m.pdopt")))
    _train(b, ob, batches[2:])
    for (k, va), (_, vb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert torch.allclose(va, vb, atol=1e-6), k


def test_checkpoint_loader_refuses_code(tmp_path):
    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))

    p = tmp_path / "evil.pdparams"
    p.write_bytes(pickle.dumps({"w": Evil()}))
    with pytest.raises(pickle.UnpicklingError):
        paddle.load(str(p))


def test_bf16_roundtrip(tmp_path):
    sd = {"w": torch.randn(3, 4).to(torch.bfloat16), "n": {"x": torch.arange(3)}}
    paddle.save(sd, str(tmp_path / "b.pdparams"))
    r = paddle.load(str(tmp_path / "b.pdparams"))
    assert r["w"].dtype == torch.bfloat16 and torch.equal(r["w"], sd["w"]) and torch.equal(r["n"]["x"], sd["n"]["x"])


def test_adam_matches_reference_formula():
    torch.manual_seed(0)
    w0 = torch.randn(5)
    gs = [torch.randn(5) for _ in range(4)]
    p = nn.Linear(5, 1).weight  # any ParamBase
    p.data = w0.clone()
    opt = paddle.optimizer.Adam(learning_rate=0.1, beta1=0.8, beta2=0.9, epsilon=1e-3, parameters=[p])
    m = v = torch.zeros(5)
    w = w0.clone()
    for t, g in enumerate(gs, 1):
        p.grad = g.clone()
        opt.step()
        m = 0.8 * m + 0.2 * g
        v = 0.9 * v + 0.1 * g * g
        lr_t = 0.1 * math.sqrt(1 - 0.9 ** t) / (1 - 0.8 ** t)
        w = w - lr_t * m / (v.sqrt() + 1e-3)  # reference adam_op.h:80-84
    assert torch.allclose(p.detach(), w, atol=1e-6)


def test_momentum_and_l2decay():
    p = nn.Linear(3, 1).weight
    p.data = torch.ones(3)
    opt = paddle.optimizer.Momentum(learning_rate=0.1, momentum=0.9, parameters=[p],
                                    weight_decay=paddle.optimizer.L2Decay(0.5))
    vel = torch.zeros(3)
    w = torch.ones(3)
    for _ in range(3):
        g = torch.full((3,), 0.2)
        p.grad = g.clone()
        opt.step()
        gg = g + 0.5 * w
        vel = 0.9 * vel + gg
        w = w - 0.1 * vel
    assert torch.allclose(p.detach(), w, atol=1e-6)


def test_lr_schedulers():
    lr = paddle.optimizer.lr
    s = lr.StepDecay(1.0, step_size=2, gamma=0.1)
    vals = []
    for _ in range(5):
        vals.append(s())
        s.step()
    assert np.allclose(vals, [1, 1, 0.1, 0.1, 0.01])
    c = lr.CosineAnnealingDecay(1.0, T_max=10)
    for _ in range(5):
        c.step()
    assert abs(c() - 0.5) < 1e-6
    w = lr.LinearWarmup(0.5, warmup_steps=4, start_lr=0.0, end_lr=0.5)
    seen = []
    for _ in range(6):
        seen.append(w())
        w.step()
    assert np.allclose(seen, [0, 0.125, 0.25, 0.375, 0.5, 0.5])
    pw = lr.PiecewiseDecay([2, 4], [1.0, 0.5, 0.1])
    got = []
    for _ in range(5):
        got.append(pw())
        pw.step()
    assert got == [1.0, 1.0, 0.5, 0.5, 0.1]


def test_grad_clip_global_norm():
    a = torch.tensor([3.0, 0.0], requires_grad=True)
    b = torch.tensor([4.0], requires_grad=True)
    (a.sum() * 0).backward()
    a.grad = torch.tensor([3.0, 0.0])
    b.grad = torch.tensor([4.0])
    paddle.nn.ClipGradByGlobalNorm(1.0)([(a, a.grad), (b, b.grad)])
    assert torch.allclose(torch.cat([a.grad, b.grad]), torch.tensor([0.6, 0.0, 0.8]), atol=1e-5)


def test_tensor_api_signatures():
    x = paddle.arange(12).reshape([3, 4]).astype("float32")
    parts = paddle.split(x, [1, -1], axis=1)
    assert parts[1].shape == (3, 3)
    assert paddle.equal(paddle.concat(parts, axis=1), x).all()
    v, i = paddle.topk(x, 2, axis=1)
    assert i.tolist() == [[3, 2]] * 3
    g = paddle.gather_nd(x, paddle.to_tensor([[0, 1], [2, 3]]))
    assert g.tolist() == [1.0, 11.0]
    assert paddle.matmul(x, x, transpose_y=True).shape == (3, 3)
    assert paddle.unsqueeze(x, [0, 2]).shape == (1, 3, 1, 4)
    assert paddle.squeeze(paddle.zeros([1, 3, 1]), axis=0).shape == (3, 1)
    t = paddle.to_tensor([1.0, 2.0], stop_gradient=False)
    assert not t.stop_gradient and t.dtype == torch.float32
    assert paddle.sum(x, axis=[0, 1]).item() == 66.0


def test_batchnorm_momentum_semantics():
    bn = nn.BatchNorm2D(2, momentum=0.9)
    x = torch.randn(4, 2, 3, 3) + 5
    bn.train()
    bn(x)
    mean = x.mean((0, 2, 3))
    assert torch.allclose(bn._mean, 0.1 * mean, atol=1e-5)


def test_conv_nhwc_matches_nchw():
    paddle.seed(0)
    c = nn.Conv2D(3, 8, 3, padding=1)
    x = torch.randn(2, 3, 9, 9)
    y1 = c(x)
    c2 = nn.Conv2D(3, 8, 3, padding=1, data_format="NHWC")
    c2.set_state_dict(c.state_dict())
    y2 = c2(x.permute(0, 2, 3, 1))
    assert torch.allclose(y1, y2.permute(0, 3, 1, 2), atol=1e-5)
    r = paddle.vision.models.resnet18(num_classes=5, data_format="NHWC")
    assert r(torch.randn(2, 32, 32, 3)).shape == (2, 5)


def test_multihead_attention_fast_path_matches_masked():
    paddle.seed(0)
    mha = nn.MultiHeadAttention(32, 4)
    x = torch.randn(2, 7, 32)
    causal = torch.ones(7, 7, dtype=torch.bool).tril()
    a = mha(x, is_causal=True)
    b = mha(x, attn_mask=causal)
    assert torch.allclose(a, b, atol=1e-5)
    enc = nn.TransformerEncoder(nn.TransformerEncoderLayer(32, 4, 64, dropout=0.0), 2)
    assert enc(x).shape == x.shape


def test_rnn_layers():
    lstm = nn.LSTM(8, 16, num_layers=2, direction="bidirect")
    out, (h, c) = lstm(torch.randn(3, 5, 8))
    assert out.shape == (3, 5, 32) and h.shape == (4, 3, 16)
    assert "weight_ih_l0_reverse" in lstm.state_dict()
    gru = nn.GRU(8, 16)
    o, h = gru(torch.randn(3, 5, 8), sequence_length=torch.tensor([5, 3, 2]))
    assert o.shape == (3, 5, 16)


def test_dataloader_workers_preserve_order():
    ds = paddle.io.TensorDataset([torch.arange(40).float().reshape(20, 2), torch.arange(20)])
    a = [b[1].tolist() for b in paddle.io.DataLoader(ds, batch_size=3, num_workers=0)]
    b = [b[1].tolist() for b in paddle.io.DataLoader(ds, batch_size=3, num_workers=3)]
    assert a == b and len(a) == 7
    s = paddle.io.DistributedBatchSampler(ds, batch_size=4, num_replicas=2, rank=1)
    idx = [i for bb in s for i in bb]
    assert idx == list(range(1, 20, 2))


def test_hapi_model_fit_evaluate(tmp_path):
    paddle.seed(2)
    net = nn.Sequential(nn.Flatten(), nn.Linear(784, 32), nn.ReLU(), nn.Linear(32, 10))
    model = paddle.Model(net)
    model.prepare(paddle.optimizer.Adam(1e-3, parameters=net.parameters()), nn.CrossEntropyLoss(),
                  paddle.metric.Accuracy())
    ds = paddle.vision.datasets.MNIST(mode="train", num_samples=256)
    hist = model.fit(ds, batch_size=32, epochs=3, verbose=0)
    assert hist[-1]["loss"] < hist[0]["loss"]
    res = model.evaluate(ds, batch_size=64, verbose=0)
    assert res["acc"] > 0.3
    model.save(str(tmp_path / "ck"))
    model.load(str(tmp_path / "ck"))


def test_grad_scaler_and_autocast():
    net = nn.Linear(4, 2)
    opt = paddle.optimizer.SGD(0.1, parameters=net.parameters())
    sc = paddle.amp.GradScaler(init_loss_scaling=1024.0)
    with paddle.amp.auto_cast():
        loss = net(torch.randn(3, 4)).float().pow(2).mean()
    sc.scale(loss).backward()
    sc.step(opt)
    sc.update()
    assert sc.get_loss_scaling() == 1024.0


def test_dygraph_1x_api():
    from paddle_amd import dygraph

    with dygraph.guard(paddle.CPUPlace()):
        x = dygraph.to_variable(np.ones((2, 1, 8, 8), "float32"))
        conv = dygraph.Conv2D(1, 4, 3, act="relu")
        pool = dygraph.Pool2D(2, "max", 2)
        fc = dygraph.FC("fc", size=3)
        y = fc(pool(conv(x)))
        assert y.shape == (2, 3)
