"""NHWC bf16 conv / batch-norm / pooling kernels (ops/conv.py) against plain PyTorch
fp32 references of the same ops (inputs rounded to bf16 first)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
dev = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


CONV_CASES = [
    # N, H, W, C, Cout, k, stride, pad, dil
    (2, 14, 14, 64, 64, 1, 1, 0, 1),
    (2, 14, 14, 64, 128, 3, 1, 1, 1),
    (2, 15, 13, 64, 64, 3, 2, 1, 1),
    (4, 8, 8, 128, 256, 1, 2, 0, 1),
    (2, 12, 12, 64, 64, 3, 1, 2, 2),
    (2, 32, 32, 3, 64, 7, 2, 3, 1),      # stem: C = 3 -> im2col path
    (1, 9, 9, 192, 72, 3, 1, 1, 1),
]


@pytest.mark.parametrize("N,H,W,C,Co,k,s,p,d", CONV_CASES)
def test_conv2d_nhwc_fwd_bwd(N, H, W, C, Co, k, s, p, d):
    from paddle_amd.ops import conv

    g = torch.Generator(device=dev).manual_seed(N * 100 + C + Co + k)
    x = torch.randn(N, H, W, C, generator=g, device=dev).to(torch.bfloat16)
    w = (torch.randn(Co, C, k, k, generator=g, device=dev) / (C * k * k) ** 0.5).to(torch.bfloat16)
    assert conv.supported_conv(x, w, s, p, d, 1)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_()
    wr = w.float().requires_grad_()
    yr = F.conv2d(xr, wr, None, s, p, d)
    xt = x.clone().requires_grad_()
    wt = w.clone().requires_grad_()
    y = conv.conv2d_nhwc(xt, wt, None, s, p, d)
    assert y.shape == yr.permute(0, 2, 3, 1).shape
    assert _rel(y, yr.permute(0, 2, 3, 1)) < 1e-2
    dy = torch.randn(y.shape, generator=g, device=dev).to(torch.bfloat16)
    yr.backward(dy.float().permute(0, 3, 1, 2))
    y.backward(dy)
    assert _rel(xt.grad, xr.grad.permute(0, 2, 3, 1)) < 2e-2
    assert _rel(wt.grad, wr.grad) < 2e-2


def test_conv2d_nhwc_bias():
    from paddle_amd.ops import conv

    x = torch.randn(2, 8, 8, 64, device=dev).to(torch.bfloat16)
    w = (torch.randn(128, 64, 3, 3, device=dev) * 0.05).to(torch.bfloat16)
    b = torch.randn(128, device=dev).to(torch.bfloat16)
    y = conv.conv2d_nhwc(x, w, b, 1, 1)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float(), b.float(), 1, 1).permute(0, 2, 3, 1)
    assert _rel(y, ref) < 1e-2


@pytest.mark.parametrize("C,relu", [(64, False), (64, True), (256, True), (2048, False), (24, True)])
def test_batch_norm_nhwc_train(C, relu):
    from paddle_amd.ops import conv

    g = torch.Generator(device=dev).manual_seed(C)
    x = (torch.randn(4, 7, 9, C, generator=g, device=dev) * 3 + 1.5).to(torch.bfloat16)
    w = torch.rand(C, generator=g, device=dev) + 0.5
    b = torch.randn(C, generator=g, device=dev)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    rm2, rv2 = rm.clone(), rv.clone()
    xt = x.clone().requires_grad_()
    wt, bt = w.clone().requires_grad_(), b.clone().requires_grad_()
    y = conv.batch_norm_nhwc_train(xt, wt, bt, rm, rv, momentum=0.9, eps=1e-5, relu=relu)
    xr = x.float().requires_grad_()
    wr, br = w.clone().requires_grad_(), b.clone().requires_grad_()
    yr = F.batch_norm(xr.reshape(-1, C), rm2, rv2, wr, br, True, 0.1, 1e-5).reshape(x.shape)
    if relu:
        yr = torch.relu(yr)
    assert _rel(y, yr) < 1e-2
    assert torch.allclose(rm, rm2, atol=1e-3, rtol=1e-3) and torch.allclose(rv, rv2, atol=1e-3, rtol=1e-3)
    dy = torch.randn(x.shape, generator=g, device=dev).to(torch.bfloat16)
    y.backward(dy)
    yr.backward(dy.float())
    assert _rel(xt.grad, xr.grad) < 2e-2
    assert _rel(wt.grad, wr.grad) < 1e-2 and _rel(bt.grad, br.grad) < 1e-2


def test_max_pool_and_gap_nhwc():
    from paddle_amd.ops import conv

    x = torch.randn(2, 17, 17, 64, device=dev).to(torch.bfloat16)
    xt = x.clone().requires_grad_()
    y = conv.max_pool2d_nhwc(xt, 3, 2, 1)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_()
    yr = F.max_pool2d(xr, 3, 2, 1)
    assert torch.equal(y.float(), yr.permute(0, 2, 3, 1))
    dy = torch.randn(y.shape, device=dev).to(torch.bfloat16)
    y.backward(dy)
    yr.backward(dy.float().permute(0, 3, 1, 2))
    assert _rel(xt.grad, xr.grad.permute(0, 2, 3, 1)) < 1e-2
    xt2 = x.clone().requires_grad_()
    ga = conv.global_avg_pool_nhwc(xt2)
    assert _rel(ga.reshape(2, 64), x.float().mean((1, 2))) < 1e-2
    ga.sum().backward()
    assert torch.allclose(xt2.grad.float(), torch.full_like(x.float(), 1 / 289), rtol=1e-2)


def test_resnet_native_matches_torch_path():
    """NHWC bf16 ResNet-50 (small input): loss and first-conv weight gradient through
    the native conv/BN/pool kernels vs an fp32 reference of the same weights; the
    native bf16 error must be no worse than the ATen/MIOpen bf16 error (x2 margin)."""
    import copy

    import paddle_amd as paddle
    from paddle_amd.ops import conv
    from paddle_amd.ops import gemm as G

    paddle.seed(0)
    torch.manual_seed(0)
    base = paddle.vision.models.resnet50(num_classes=10, data_format="NHWC").to(dev)
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(8, 64, 64, 3, generator=g, device=dev)
    y = torch.randint(0, 10, (8,), generator=g, device=dev)

    def run(dtype, native):
        G.set_enabled(native)
        conv.set_enabled(native)
        try:
            m = copy.deepcopy(base).to(dtype)
            logits = m(x.to(dtype)).float()
            loss = F.cross_entropy(logits, y)
            loss.backward()
            l1, l4 = list(m.layer1.children()), list(m.layer4.children())
            grads = [m.conv1.weight.grad, l1[0].conv2.weight.grad, l4[-1].conv3.weight.grad,
                     l4[-1].bn3.weight.grad, m.fc.weight.grad]
            return loss.item(), [t.float().flatten() for t in grads], logits.detach()
        finally:
            G.set_enabled(True)
            conv.set_enabled(True)

    l32, g32, z32 = run(torch.float32, False)
    la, ga, za = run(torch.bfloat16, False)
    ln, gn, zn = run(torch.bfloat16, True)
    # a random-init bf16 ResNet-50 carries ~30 % relative logit error on BOTH paths
    # (measured: native 0.291, ATen/MIOpen 0.298), so the scalar loss gap to fp32 is
    # noise of either sign; compare the logit error itself, plus a loose loss bound
    rel = lambda a, b: ((a - b).norm() / b.norm()).item()  # noqa: E731
    en, ea = rel(zn, z32), rel(za, z32)
    assert en <= 1.25 * ea + 0.02, (en, ea)
    assert abs(ln - l32) <= 0.15, (ln, la, l32)
    cos = lambda a, b: (a @ b / (a.norm() * b.norm())).item()  # noqa: E731
    # (a random-init bf16 ResNet-50's stem gradient is far from fp32 on either path;
    # the criterion is relative: native no worse than the vendor bf16 path)
    for i, (n_, a_, r_) in enumerate(zip(gn, ga, g32)):
        cn, ca = cos(n_, r_), cos(a_, r_)
        print(f"grad {i}: cos(native, fp32) = {cn:.4f}  cos(aten bf16, fp32) = {ca:.4f}")
        assert cn >= ca - 0.05, (i, cn, ca)


SN_CASES = [
    # N, H, W, C, Cout, k, stride, pad  (64-channel-tile kernel, csrc/kernels/convsn.hip)
    (2, 14, 14, 64, 64, 3, 1, 1),
    (3, 9, 11, 128, 128, 1, 1, 0),
    (2, 15, 13, 64, 48, 3, 2, 1),
    (1, 7, 7, 192, 200, 3, 1, 1),
]


@pytest.mark.parametrize("N,H,W,C,Co,k,s,p", SN_CASES)
def test_conv_sn_matches_reference_and_emits_bn_stats(N, H, W, C, Co, k, s, p):
    from paddle_amd.ops import conv

    g = torch.Generator(device=dev).manual_seed(7 * C + Co)
    x = torch.randn(N, H, W, C, generator=g, device=dev).to(torch.bfloat16)
    w = (torch.randn(Co, C, k, k, generator=g, device=dev) / (C * k * k) ** 0.5).to(torch.bfloat16)
    shift = torch.randn(Co, generator=g, device=dev) * 0.1
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float(), None, s, p).permute(0, 2, 3, 1)
    old = conv._SN_MAX[0]
    try:
        conv._SN_MAX[0] = 0
        yw = conv.conv2d_nhwc(x, w, None, s, p)
        conv._SN_MAX[0] = 1 << 16
        st = {"shift": shift}
        ys = conv.conv2d_nhwc(x, w, None, s, p, stats=st)
    finally:
        conv._SN_MAX[0] = old
    assert _rel(ys, ref) < 1e-2 and _rel(yw, ref) < 1e-2
    assert st.get("part") is not None
    G = st["G"]
    part = st["part"].view(G, 2, Co).double()
    d = ys.double().reshape(-1, Co) - shift.double()
    torch.testing.assert_close(part[:, 0].sum(0), d.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(part[:, 1].sum(0), (d * d).sum(0), rtol=1e-4, atol=1e-2)
    # the 256-wide-tile kernel emits the same statistics from its staged epilogue
    try:
        conv._SN_MAX[0] = 0
        st2 = {"shift": shift}
        yw2 = conv.conv2d_nhwc(x, w, None, s, p, stats=st2)
    finally:
        conv._SN_MAX[0] = old
    assert torch.equal(yw2, yw) and st2.get("part") is not None and st2["G"] == G
    part2 = st2["part"].view(G, 2, Co).double()
    d2 = yw2.double().reshape(-1, Co) - shift.double()
    torch.testing.assert_close(part2[:, 0].sum(0), d2.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(part2[:, 1].sum(0), (d2 * d2).sum(0), rtol=1e-4, atol=1e-2)


def test_conv_bn_relu_fused_stats_match_unfused():
    """ResNet bottleneck entry: conv -> BN(+ReLU) with the statistics from the conv
    epilogue equals the two-pass BN (outputs, running statistics, gradients)."""
    import paddle_amd as paddle
    from paddle_amd import nn
    from paddle_amd.vision import models as VM

    paddle.seed(3)
    c = nn.Conv2D(64, 64, 3, padding=1, bias_attr=False, data_format="NHWC").to(dev).to(torch.bfloat16)
    bn = nn.BatchNorm2D(64, data_format="NHWC").to(dev)
    g = torch.Generator(device=dev).manual_seed(5)
    x = (torch.randn(4, 16, 16, 64, generator=g, device=dev) + 0.5).to(torch.bfloat16)
    states = []
    outs = []
    for fused in (False, True):
        bn._mean.zero_()
        bn._variance.fill_(1.0)
        for prm in list(c.parameters()) + list(bn.parameters()):
            prm.grad = None
        xt = x.clone().requires_grad_()
        y = VM._conv_bn_relu(c, bn, xt) if fused else VM._bn_relu(bn, c(xt))
        y.float().pow(2).sum().backward()
        outs.append((y.detach().float(), xt.grad.float(), c.weight.grad.float(), bn.weight.grad.float()))
        states.append((bn._mean.clone(), bn._variance.clone()))
    for a, b in zip(outs[0], outs[1]):
        assert _rel(b, a) < 2e-2
    torch.testing.assert_close(states[1][0], states[0][0], rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(states[1][1], states[0][1], rtol=1e-3, atol=1e-4)


def test_bottleneck_residual_grad_accumulated_in_dgrad_epilogue():
    """The block input's gradient = residual branch (BN3 backward's dres) + conv1's
    dX: with the engine's accumulate-into protocol conv1's dgrad sums onto dres in its
    epilogue (no add kernel); gradients must equal the plain engine sum."""
    import paddle_amd as paddle
    from paddle_amd.autograd import engine as E
    from paddle_amd.vision.models import BottleneckBlock

    paddle.seed(11)
    blk = BottleneckBlock(256, 64, data_format="NHWC").to(dev).to(torch.bfloat16)
    g = torch.Generator(device=dev).manual_seed(2)
    x0 = torch.randn(4, 14, 14, 256, generator=g, device=dev).to(torch.bfloat16)
    res = []
    for on in (False, True):
        E._ACCUM_INTO[0] = on
        try:
            for q in blk.parameters():
                q.grad = None
            x = paddle.to_tensor(x0.clone(), stop_gradient=False)
            y = blk(x)
            (y.astype("float32") ** 2).sum().backward()
            res.append((x.grad.float().clone(), blk.conv1.weight.grad.float().clone()))
        finally:
            E._ACCUM_INTO[0] = True
    assert _rel(res[1][0], res[0][0]) < 1e-2
    assert _rel(res[1][1], res[0][1]) < 1e-2


BNB_CASES = [
    # N, H, W, C, Cout, k, stride, pad, y-mask, accumulate  (C <= 128: 64-channel tiles; else 256-wide GEMM)
    (2, 14, 14, 64, 64, 3, 1, 1, False, False),
    (2, 15, 13, 64, 128, 3, 2, 1, True, False),
    (3, 9, 11, 128, 64, 1, 1, 0, False, True),
    (2, 8, 8, 256, 64, 1, 1, 0, False, False),
    (4, 8, 8, 256, 128, 1, 2, 0, True, True),
]


@pytest.mark.parametrize("N,H,W,C,Co,k,s,p,ymask,acc", BNB_CASES)
def test_dgrad_epilogue_emits_bn_backward_stats(N, H, W, C, Co, k, s, p, ymask, acc):
    """The conv data gradient with BatchNorm-backward statistics (pa_conv_sn_bnbwd /
    pa_conv_gemm_bnbwd): dX unchanged, and the partials sum to sum(g), sum(g (x - mean))
    with g = the stored dX under the ReLU mask (from y, or recomputed from x)."""
    from paddle_amd.ops import conv

    g = torch.Generator(device=dev).manual_seed(N * 31 + C + Co + k)
    OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = torch.randn(N, OH, OW, Co, generator=g, device=dev).to(torch.bfloat16)
    w = (torch.randn(Co, C, k, k, generator=g, device=dev) / (Co * k * k) ** 0.5).to(torch.bfloat16)
    xb = (torch.randn(N, H, W, C, generator=g, device=dev) + 0.3).to(torch.bfloat16)
    mean = torch.randn(C, generator=g, device=dev) * 0.2
    rstd = torch.rand(C, generator=g, device=dev) + 0.5
    bw = torch.rand(C, generator=g, device=dev) + 0.5
    bb = torch.randn(C, generator=g, device=dev) * 0.3
    yb = torch.randn(N, H, W, C, generator=g, device=dev).to(torch.bfloat16) if ymask else None
    prev = torch.randn(N, H, W, C, generator=g, device=dev).to(torch.bfloat16)
    plain = conv._conv_dgrad(dy, w, (N, H, W, C), (s, s), (p, p), (1, 1),
                             into=prev.clone() if acc else None)
    bnb = {"x": xb, "y": yb, "mean": mean, "rstd": rstd, "w": bw, "b": bb, "wdt": 0, "relu": 1}
    dx = conv._conv_dgrad(dy, w, (N, H, W, C), (s, s), (p, p), (1, 1), into=prev.clone() if acc else None, bnb=bnb)
    assert torch.equal(dx, plain)
    bp = getattr(dx, "_pa_bnpart", None)
    assert bp is not None and bp[2] is mean
    G = bp[1]
    part = bp[0].view(G, 2, C).double().sum(0)
    xf = xb.double().reshape(-1, C)
    if ymask:
        keep = yb.double().reshape(-1, C) > 0
    else:
        sc = rstd.double() * bw.double()
        keep = (xf * sc + (bb.double() - mean.double() * sc)) > 0
    gg = dx.double().reshape(-1, C) * keep
    torch.testing.assert_close(part[0], gg.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(part[1], (gg * (xf - mean.double())).sum(0), rtol=1e-4, atol=1e-2)


def test_resnet_blocks_bn_backward_stats_match_two_pass():
    """Two bottleneck blocks (the second strided with a projection shortcut, so the
    first block's output has two consuming convs and a residual-ReLU mask): every
    gradient with the BN backward statistics taken in the consuming dgrad epilogues
    (FLAGS_conv_bn_bwd_stats=1, off by default: measured slower) equals the
    separate-reduction path, and the epilogue path is the one taken."""
    import paddle_amd as paddle
    from paddle_amd import nn
    from paddle_amd.ops import conv
    from paddle_amd.ops import _native as N_
    from paddle_amd.vision.models import BottleneckBlock

    paddle.seed(13)
    ds = nn.Sequential(nn.Conv2D(256, 512, 1, stride=2, bias_attr=False, data_format="NHWC"),
                       nn.BatchNorm2D(512, data_format="NHWC"))
    net = nn.Sequential(BottleneckBlock(256, 64, data_format="NHWC"),
                        BottleneckBlock(256, 128, stride=2, downsample=ds, data_format="NHWC")).to(dev)
    net = net.to(torch.bfloat16)
    g = torch.Generator(device=dev).manual_seed(4)
    x0 = torch.randn(4, 16, 16, 256, generator=g, device=dev).to(torch.bfloat16)
    real_call = N_.call
    saved = conv._BNB[0]
    res = []
    for on in (False, True):
        used = []

        def counting(name, *a, **k):
            if name == "pa_bn_bwd_part":
                used.append(name)
            return real_call(name, *a, **k)

        conv._BNB[0] = on
        N_.call = counting
        try:
            for q in net.parameters():
                q.grad = None
            x = paddle.to_tensor(x0.clone(), stop_gradient=False)
            y = net(x)
            (y.astype("float32") ** 2).mean().backward()
            res.append([x.grad.float().clone()] + [q.grad.float().clone() for q in net.parameters()])
        finally:
            N_.call = real_call
            conv._BNB[0] = saved
        # 5 ReLU BatchNorms whose output feeds a convolution (bn1, bn2 of both blocks,
        # bn3 of the first); the last block's bn3 and the shortcut BN have no conv consumer
        assert len(used) == (5 if on else 0), used
    for a, b in zip(res[0], res[1]):
        assert _rel(b, a) < 2e-2
