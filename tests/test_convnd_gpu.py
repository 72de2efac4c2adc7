"""Channel-first conv / transposed conv / pooling / unpool / maxout kernels
(csrc/kernels/convnd.hip via ops/convnd.py) against fp64 PyTorch references of
the same ops: forward and both gradients, odd sizes, strides, paddings,
dilations, groups (incl. depthwise), 2-D and 3-D; the exact-fp32 MFMA GEMM on
strided / batched / atomic forms."""
import pytest
import torch
import torch.nn.functional as F

from paddle_amd.ops import convnd as C

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (37, 129, 65), (128, 128, 16), (300, 70, 513)])
def test_sgemm_forms(M, N, K):
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    A = torch.randn(3, 2, M, K, generator=g, device=DEV)
    B = torch.randn(3, 2, K, N, generator=g, device=DEV)
    ref = (A.double() @ B.double())
    # row-major A and B, batch (3, 2) on z1 x z2, bias per row (+ per z2 offset)
    Cc = torch.empty(3, 2, M, N, device=DEV)
    bias = torch.randn(2, M, generator=g, device=DEV)
    C.sgemm(A, K, 1, B, N, 1, Cc, N, M, N, K, Z1=3, Z2=2, bs1=(2 * M * K, 2 * K * N, 2 * M * N),
            bs2=(M * K, K * N, M * N), bias=bias, bs_bias2=M)
    assert _rel(Cc, ref + bias.double()[None, :, :, None]) < 1e-6
    # transposed operands (A given as [K, M], B as [N, K]), beta = 1
    At = A[0, 0].t().contiguous()
    Bt = B[0, 0].t().contiguous()
    C0 = torch.randn(M, N, generator=g, device=DEV)
    C1 = C0.clone()
    C.sgemm(At, 1, M, Bt, 1, K, C1, N, M, N, K, alpha=0.5, beta=1.0)
    assert _rel(C1, 0.5 * ref[0, 0] + C0.double()) < 1e-6
    # k-batch (sum of the 3 z1 products in registers) and atomic split over z2
    Ca = torch.zeros(M, N, device=DEV)
    C.sgemm(A, K, 1, B, N, 1, Ca, N, M, N, K, Z1=1, Z2=2, bs2=(M * K, K * N, 0), kb=3, kbA=2 * M * K,
            kbB=2 * K * N, atomic=True)
    assert _rel(Ca, ref.sum((0, 1))) < 1e-6


CONV2D = [
    # (N, C, H, W, Cout, k, stride, pad, dil, groups, bias)
    (2, 3, 9, 7, 5, (3, 3), (1, 1), (1, 1), (1, 1), 1, True),
    (3, 8, 11, 10, 12, (3, 2), (2, 1), (0, 1), (1, 2), 4, False),
    (2, 16, 8, 8, 16, (3, 3), (1, 1), (1, 1), (1, 1), 16, True),   # depthwise
    (1, 64, 14, 14, 128, (1, 1), (2, 2), (0, 0), (1, 1), 1, False),
    (4, 5, 6, 13, 7, (5, 5), (3, 2), (2, 2), (1, 1), 1, True),
    (3, 8, 5, 7, 12, (1, 1), (1, 1), (0, 0), (1, 1), 2, True),     # pointwise: no vol2col
    (2, 16, 9, 9, 32, (1, 1), (1, 1), (0, 0), (1, 1), 1, False),
]


@pytest.mark.parametrize("cfg", CONV2D)
def test_conv2d_fwd_bwd(cfg):
    Nn, Ci, H, W, Co, k, s, p, d, G, has_b = cfg
    g = torch.Generator().manual_seed(sum(cfg[:5]))
    x = torch.randn(Nn, Ci, H, W, generator=g, dtype=torch.float64)
    w = torch.randn(Co, Ci // G, *k, generator=g, dtype=torch.float64) * 0.3
    b = torch.randn(Co, generator=g, dtype=torch.float64) if has_b else None
    xr, wr = x.clone().requires_grad_(), w.clone().requires_grad_()
    br = b.clone().requires_grad_() if has_b else None
    ref = F.conv2d(xr, wr, br, s, p, d, G)
    xd, wd = x.float().to(DEV).requires_grad_(), w.float().to(DEV).requires_grad_()
    bd = b.float().to(DEV).requires_grad_() if has_b else None
    assert C.supported_conv(xd, wd, G)
    y = C.conv_nd(xd, wd, bd, s, p, d, G)
    assert y.shape == ref.shape
    assert _rel(y, ref) < 1e-5
    gy = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    ref.backward(gy)
    y.backward(gy.float().to(DEV))
    assert _rel(xd.grad, xr.grad) < 1e-5
    assert _rel(wd.grad, wr.grad) < 1e-5
    if has_b:
        assert _rel(bd.grad, br.grad) < 1e-5


@pytest.mark.parametrize("cfg", [
    (2, 3, (5, 6, 7), 4, (3, 3, 3), (1, 1, 1), (1, 1, 1), (1, 1, 1), 1),
    (1, 4, (4, 9, 8), 6, (2, 3, 2), (2, 2, 1), (0, 1, 1), (1, 1, 2), 2),
])
def test_conv3d_fwd_bwd(cfg):
    Nn, Ci, sp, Co, k, s, p, d, G = cfg
    g = torch.Generator().manual_seed(3)
    x = torch.randn(Nn, Ci, *sp, generator=g, dtype=torch.float64)
    w = torch.randn(Co, Ci // G, *k, generator=g, dtype=torch.float64) * 0.3
    xr, wr = x.clone().requires_grad_(), w.clone().requires_grad_()
    ref = F.conv3d(xr, wr, None, s, p, d, G)
    xd, wd = x.float().to(DEV).requires_grad_(), w.float().to(DEV).requires_grad_()
    y = C.conv_nd(xd, wd, None, s, p, d, G)
    assert _rel(y, ref) < 1e-5
    gy = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    ref.backward(gy)
    y.backward(gy.float().to(DEV))
    assert _rel(xd.grad, xr.grad) < 1e-5
    assert _rel(wd.grad, wr.grad) < 1e-5


@pytest.mark.parametrize("cfg", [
    (2, 4, (5, 6), 3, (3, 3), (2, 2), (1, 1), (1, 1), 1, (0, 0)),
    (1, 6, (4, 7), 2, (4, 3), (2, 3), (1, 0), (1, 1), 3, (1, 2)),
    (2, 2, (3, 4, 3), 3, (3, 2, 3), (2, 1, 2), (1, 0, 1), (1, 2, 1), 1, (1, 0, 0)),
])
def test_conv_transpose_fwd_bwd(cfg):
    Nn, Ci, sp, Cog, k, s, p, d, G, op = cfg
    g = torch.Generator().manual_seed(4)
    x = torch.randn(Nn, Ci, *sp, generator=g, dtype=torch.float64)
    w = torch.randn(Ci, Cog, *k, generator=g, dtype=torch.float64) * 0.3
    xr, wr = x.clone().requires_grad_(), w.clone().requires_grad_()
    fn = F.conv_transpose2d if len(sp) == 2 else F.conv_transpose3d
    ref = fn(xr, wr, None, s, p, op, G, d)
    xd, wd = x.float().to(DEV).requires_grad_(), w.float().to(DEV).requires_grad_()
    y = C.conv_transpose_nd(xd, wd, s, p, d, G, op)
    assert y.shape == ref.shape
    assert _rel(y, ref) < 1e-5
    gy = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    ref.backward(gy)
    y.backward(gy.float().to(DEV))
    assert _rel(xd.grad, xr.grad) < 1e-5
    assert _rel(wd.grad, wr.grad) < 1e-5


def test_conv_bf16_input_computes_in_fp32():
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 8, 10, 10, generator=g).to(torch.bfloat16)
    w = torch.randn(8, 8, 3, 3, generator=g).to(torch.bfloat16)
    y = C.conv_nd(x.to(DEV), w.to(DEV), None, 1, 1, 1, 1)
    assert y.dtype == torch.bfloat16
    ref = F.conv2d(x.double(), w.double(), None, 1, 1)
    assert _rel(y, ref) < 1e-2


def _paddle_avg_ref(x, k, s, p, exclusive, ceil):
    """pooling.cu KernelPool{2,3}D avg semantics (clamped window, divisor = clamped
    size if exclusive else the full kernel), computed in fp64 by loops over windows."""
    nd = x.dim() - 2
    sp = x.shape[2:]
    osp = [C.pool_out(sp[i], k[i], s[i], p[i], ceil) for i in range(nd)]
    out = torch.zeros(tuple(x.shape[:2]) + tuple(osp), dtype=torch.float64)
    import itertools
    for o in itertools.product(*[range(v) for v in osp]):
        lo = [max(o[i] * s[i] - p[i], 0) for i in range(nd)]
        hi = [min(o[i] * s[i] - p[i] + k[i], sp[i]) for i in range(nd)]
        sl = (slice(None), slice(None)) + tuple(slice(lo[i], hi[i]) for i in range(nd))
        win = x[sl]
        cnt = 1
        for i in range(nd):
            cnt *= (hi[i] - lo[i]) if exclusive else k[i]
        out[(slice(None), slice(None)) + tuple(o)] = win.sum(tuple(range(2, 2 + nd))) / cnt if cnt else 0
    return out


@pytest.mark.parametrize("shape,k,s,p,exclusive,ceil", [
    ((2, 3, 9, 8), (3, 3), (2, 2), (1, 1), True, False),
    ((2, 3, 9, 8), (3, 2), (2, 3), (1, 0), False, True),
    ((1, 2, 5, 6, 7), (2, 3, 2), (2, 2, 2), (0, 1, 1), True, True),
    ((1, 2, 5, 6, 7), (3, 3, 3), (1, 2, 2), (1, 1, 0), False, False),
])
def test_avg_pool_fwd_bwd(shape, k, s, p, exclusive, ceil):
    g = torch.Generator().manual_seed(6)
    x = torch.randn(*shape, generator=g, dtype=torch.float64)
    xr = x.clone().requires_grad_()
    ref = _paddle_avg_ref(xr, k, s, p, exclusive, ceil)
    xd = x.float().to(DEV).requires_grad_()
    y = C.pool_nd(xd, "avg", k, s, p, exclusive, ceil)
    assert y.shape == ref.shape
    assert _rel(y, ref) < 1e-6
    gy = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    ref.backward(gy)
    y.backward(gy.float().to(DEV))
    assert _rel(xd.grad, xr.grad) < 1e-6


@pytest.mark.parametrize("shape,k,s,p", [
    ((2, 3, 9, 8), (3, 3), (2, 2), (1, 1)),
    ((2, 4, 7, 10), (2, 4), (1, 3), (0, 2)),
    ((1, 2, 6, 7, 5), (2, 3, 2), (2, 2, 1), (1, 1, 0)),
])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_max_pool_with_index_fwd_bwd(shape, k, s, p, dtype):
    g = torch.Generator().manual_seed(7)
    x = torch.randn(*shape, generator=g).to(dtype).double()
    xr = x.clone().requires_grad_()
    fn = F.max_pool2d if len(shape) == 4 else F.max_pool3d
    ref, idx = fn(xr, k, s, p, return_indices=True)
    xd = x.to(dtype).to(DEV).requires_grad_()
    y, mask = C.pool_nd(xd, "max", k, s, p, return_mask=True)
    assert torch.equal(y.double().cpu(), ref.detach())
    assert torch.equal(mask.long().cpu(), idx)
    gy = torch.randn(ref.shape, generator=g, dtype=torch.float64).to(dtype).double()
    ref.backward(gy)
    y.backward(gy.to(dtype).to(DEV))
    assert _rel(xd.grad, xr.grad) < (1e-6 if dtype == torch.float32 else 1e-2)


def test_unpool_and_maxout():
    g = torch.Generator().manual_seed(8)
    x = torch.randn(2, 3, 8, 6, generator=g)
    pooled, idx = F.max_pool2d(x, 2, 2, return_indices=True)
    pr = pooled.double().requires_grad_()
    ref = F.max_unpool2d(pr, idx, 2, 2)
    pd = pooled.to(DEV).requires_grad_()
    out = C.unpool2d(pd, idx.to(torch.int32).to(DEV), 2, 2, 0)
    assert torch.equal(out.double().cpu(), ref.detach())
    gy = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    ref.backward(gy)
    out.backward(gy.float().to(DEV))
    assert _rel(pd.grad, pr.grad) < 1e-7
    with pytest.raises(ValueError):
        C.unpool2d(pd.detach(), torch.full(idx.shape, 999, dtype=torch.int32, device=DEV), 2, 2, 0)

    x = torch.randn(2, 6, 4, 5, generator=g, dtype=torch.float64)
    xr = x.clone().requires_grad_()
    ref = xr.reshape(2, 3, 2, 4, 5).max(2).values
    xd = x.float().to(DEV).requires_grad_()
    y = C.maxout(xd, 2)
    assert torch.equal(y.double().cpu(), ref.detach().float().double())
    gy = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    ref.backward(gy)
    y.backward(gy.float().to(DEV))
    assert _rel(xd.grad, xr.grad) < 1e-7


def test_fluid_conv_pool_program_matches_cpu():
    """A Fluid conv -> pool -> conv_transpose -> fc program: forward and parameter
    gradients on CUDAPlace (convnd kernels) equal CPUPlace (ATen) within fp32."""
    import numpy as np

    import paddle_amd.fluid as fluid

    def run(place):
        main, startup = fluid.Program(), fluid.Program()
        main.random_seed = startup.random_seed = 11
        with fluid.program_guard(main, startup):
            img = fluid.layers.data("img", [3, 12, 12], dtype="float32")
            c = fluid.layers.conv2d(img, 8, 3, padding=1, act="relu", groups=1)
            pl = fluid.layers.pool2d(c, 2, "max", 2)
            c2 = fluid.layers.conv2d(pl, 8, 3, padding=1, groups=4)
            ct = fluid.layers.conv2d_transpose(c2, 4, filter_size=2, stride=2)
            pa = fluid.layers.pool2d(ct, 3, "avg", 2, pool_padding=1)
            loss = fluid.layers.mean(fluid.layers.fc(pa, 5))
            fluid.optimizer.SGD(0.1).minimize(loss)
        exe = fluid.Executor(place)
        scope = fluid.core.Scope()
        with fluid.scope_guard(scope):
            exe.run(startup)
            rs = np.random.RandomState(1)  # same initial weights on both places
            for prm in main.global_block().all_parameters():
                t = scope.find_var(prm.name).get_tensor()
                t.set((rs.randn(*np.array(t).shape) * 0.2).astype("float32"), place)
            x = np.random.RandomState(0).randn(4, 3, 12, 12).astype("float32")
            outs = [exe.run(main, feed={"img": x}, fetch_list=[loss])[0] for _ in range(3)]
            params = [np.array(scope.find_var(p.name).get_tensor()) for p in main.global_block().all_parameters()]
        return np.array(outs).ravel(), params

    lc, pc = run(fluid.CPUPlace())
    lg, pg = run(fluid.CUDAPlace(0))
    np.testing.assert_allclose(lg, lc, rtol=1e-4, atol=1e-5)
    assert len(pc) == len(pg) == 8
    for a, b in zip(pg, pc):
        np.testing.assert_allclose(a, b, rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("shape", [(4, 6, 5, 7), (16, 10), (2, 3, 4, 5, 6), (1, 8, 33, 65)])
@pytest.mark.parametrize("relu", [False, True])
def test_batch_norm_nchw_train(shape, relu):
    g = torch.Generator().manual_seed(9)
    x = torch.randn(*shape, generator=g, dtype=torch.float64) * 2 + 3
    C = shape[1]
    sc = torch.rand(C, generator=g, dtype=torch.float64) + 0.5
    bi = torch.randn(C, generator=g, dtype=torch.float64)
    rm, rv = torch.randn(C, generator=g, dtype=torch.float64), torch.rand(C, generator=g, dtype=torch.float64) + 1
    xr, sr, br = (t.clone().requires_grad_() for t in (x, sc, bi))
    dims = [0] + list(range(2, x.dim()))
    shp = [1, C] + [1] * (x.dim() - 2)
    mu, var = xr.mean(dims), xr.var(dims, unbiased=False)
    ref = (xr - mu.reshape(shp)) / torch.sqrt(var.reshape(shp) + 1e-5) * sr.reshape(shp) + br.reshape(shp)
    if relu:
        ref = torch.relu(ref)
    xd, sd, bd = (t.float().to(DEV).requires_grad_() for t in (x, sc, bi))
    y, mo, vo, sm, sv = C_bn(xd, sd, bd, rm.float().to(DEV), rv.float().to(DEV), relu)
    assert _rel(y, ref) < 1e-5
    torch.testing.assert_close(mo.double().cpu(), 0.9 * rm + 0.1 * mu.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(vo.double().cpu(), 0.9 * rv + 0.1 * var.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(sv.double().cpu(), 1 / torch.sqrt(var.detach() + 1e-5), rtol=1e-5, atol=1e-6)
    gy = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    ref.backward(gy)
    y.backward(gy.float().to(DEV))
    assert _rel(xd.grad, xr.grad) < 1e-4
    assert _rel(sd.grad, sr.grad) < 1e-5
    assert _rel(bd.grad, br.grad) < 1e-5


def C_bn(x, s, b, rm, rv, relu):
    return C.batch_norm_nchw(x, s, b, rm, rv, 0.9, 1e-5, training=True, relu=relu)


def test_batch_norm_nchw_eval_and_bf16():
    g = torch.Generator().manual_seed(10)
    x = torch.randn(3, 5, 6, 6, generator=g)
    sc, bi = torch.rand(5, generator=g) + 0.5, torch.randn(5, generator=g)
    rm, rv = torch.randn(5, generator=g), torch.rand(5, generator=g) + 1
    ref = F.batch_norm(x.double(), rm.double(), rv.double(), sc.double(), bi.double(), False, 0.0, 1e-5)
    y, mo, vo, _, _ = C.batch_norm_nchw(x.to(DEV), sc.to(DEV), bi.to(DEV), rm.to(DEV), rv.to(DEV), training=False)
    assert _rel(y, ref) < 1e-6
    assert torch.equal(mo.cpu(), rm) and torch.equal(vo.cpu(), rv)
    yb, _, _, _, _ = C.batch_norm_nchw(x.to(torch.bfloat16).to(DEV), sc.to(DEV), bi.to(DEV), rm.to(DEV), rv.to(DEV),
                                       training=False)
    assert yb.dtype == torch.bfloat16 and _rel(yb, ref) < 1e-2
    # nn layer path (2.x convention: unbiased running variance, updated in place)
    import paddle_amd as paddle

    bn = paddle.nn.BatchNorm2D(5).to(DEV)
    bn.train()
    out = bn(x.to(DEV))
    tr = torch.nn.BatchNorm2d(5, momentum=0.1, eps=1e-5).double()
    with torch.no_grad():
        tr.weight.copy_(bn.weight.double().cpu())
        tr.bias.copy_(bn.bias.double().cpu())
    ro = tr(x.double())
    assert _rel(out, ro) < 1e-5
    torch.testing.assert_close(bn._variance.double().cpu(), tr.running_var, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("shape", [((33, 70), (70, 129)), ((4, 17, 40), (40, 9)), ((3, 8, 16), (3, 16, 24)),
                                   ((128, 512), (512, 2048))])
@pytest.mark.parametrize("trans", [False, True])
def test_fluid_blas_matmul_fwd_bwd(shape, trans):
    from paddle_amd.ops import blas

    sa, sb = shape
    g = torch.Generator().manual_seed(11)
    a = torch.randn(*sa, generator=g, dtype=torch.float64)
    b = torch.randn(*sb, generator=g, dtype=torch.float64)
    ar, br = a.clone().requires_grad_(), b.clone().requires_grad_()
    ref = 0.5 * (ar @ br)
    ad = a.float().to(DEV)
    bd = b.float().to(DEV)
    if trans:  # operands handed over as transposed strided views
        ad = ad.transpose(-1, -2).contiguous().transpose(-1, -2)
        bd = bd.transpose(-1, -2).contiguous().transpose(-1, -2)
    ad.requires_grad_()
    bd.requires_grad_()
    assert blas.supported(ad, bd)
    y = blas.matmul(ad, bd, 0.5)
    assert _rel(y, ref) < 1e-6
    gy = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    ref.backward(gy)
    y.backward(gy.float().to(DEV))
    assert _rel(ad.grad, ar.grad) < 1e-6
    assert _rel(bd.grad, br.grad) < 1e-6


def test_fluid_blas_fc():
    from paddle_amd.ops import blas

    g = torch.Generator().manual_seed(12)
    x = torch.randn(37, 50, generator=g, dtype=torch.float64)
    w = torch.randn(50, 21, generator=g, dtype=torch.float64)
    b = torch.randn(21, generator=g, dtype=torch.float64)
    xr, wr, br = (t.clone().requires_grad_() for t in (x, w, b))
    ref = xr @ wr + br
    xd, wd, bd = (t.float().to(DEV).requires_grad_() for t in (x, w, b))
    y = blas.fc(xd, wd, bd)
    assert _rel(y, ref) < 1e-6
    gy = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    ref.backward(gy)
    y.backward(gy.float().to(DEV))
    for d_, r_ in ((xd, xr), (wd, wr), (bd, br)):
        assert _rel(d_.grad, r_.grad) < 1e-6


def test_conv2d_implicit_gemm_mode(monkeypatch):
    """The zero-column-buffer 2-D path (B gathered in the GEMM tile loader)."""
    monkeypatch.setattr(C, "_IMPLICIT", True)
    for cfg in CONV2D:
        test_conv2d_fwd_bwd(cfg)
