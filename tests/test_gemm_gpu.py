"""Numerics of the hand-written gfx950 MFMA GEMM (csrc/kernels/gemm.hip) against a
plain PyTorch fp32 reference of the same product, for every operand layout, both
output dtypes, accumulate, bias, batch, and shapes that are not tile multiples."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(8, 8, 8), (264, 136, 72), (520, 1032, 4104), (1024, 768, 512), (256, 256, 64), (2056, 512, 136)]


def _operand(rows_mn, K, kmaj, gen):
    # K-major: [MN, K]; MN-major: stored [K, MN]; returns (stored tensor, logical [MN, K] fp32)
    if kmaj:
        t = torch.randn(rows_mn, K, generator=gen, device="cuda").to(torch.bfloat16)
        return t, t.float()
    t = torch.randn(K, rows_mn, generator=gen, device="cuda").to(torch.bfloat16)
    return t, t.float().t()


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("a_kmaj", [True, False])
@pytest.mark.parametrize("b_kmaj", [True, False])
def test_gemm_layouts_bf16(M, N, K, a_kmaj, b_kmaj):
    from paddle_amd.ops import gemm as G

    gen = torch.Generator(device="cuda").manual_seed(M * 7 + N * 3 + K)
    a, af = _operand(M, K, a_kmaj, gen)
    b, bf = _operand(N, K, b_kmaj, gen)
    c = G.gemm(a, b, M, N, K, a_kmaj=a_kmaj, b_kmaj=b_kmaj)
    ref = af @ bf.t()
    err = (c.float() - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= 1e-2 * scale + 1e-3, (err, scale)


@pytest.mark.parametrize("M,N,K", [(264, 136, 72), (1024, 768, 4104)])
@pytest.mark.parametrize("a_kmaj,b_kmaj", [(True, False), (False, False), (True, True)])
def test_gemm_fp32_accumulate_and_bias(M, N, K, a_kmaj, b_kmaj):
    from paddle_amd.ops import gemm as G

    gen = torch.Generator(device="cuda").manual_seed(11)
    a, af = _operand(M, K, a_kmaj, gen)
    b, bf = _operand(N, K, b_kmaj, gen)
    c0 = torch.randn(M, N, generator=gen, device="cuda")
    c = c0.clone()
    G.gemm(a, b, M, N, K, a_kmaj=a_kmaj, b_kmaj=b_kmaj, out=c, accumulate=True, alpha=0.5)
    ref = c0 + 0.5 * (af @ bf.t())
    assert torch.allclose(c, ref, atol=2e-3 * K ** 0.5, rtol=1e-4), (c - ref).abs().max()
    bias = torch.randn(N, generator=gen, device="cuda").to(torch.bfloat16)
    y = G.gemm(a, b, M, N, K, a_kmaj=a_kmaj, b_kmaj=b_kmaj, bias=bias)
    ref = af @ bf.t() + bias.float()
    assert (y.float() - ref).abs().max() <= 1e-2 * ref.abs().max() + 1e-3


def test_gemm_identity_asymmetric():
    # A = I with an asymmetric B catches a transposed C write (guide §3)
    from paddle_amd.ops import gemm as G

    n = 256
    a = torch.eye(n, device="cuda", dtype=torch.bfloat16)
    b = (torch.arange(n, device="cuda")[:, None] * 3 + torch.arange(n, device="cuda")[None, :] * 0.01
         ).to(torch.bfloat16)
    c = G.matmul_nt(a, b)
    assert torch.equal(c, b.t().contiguous())


def test_gemm_batched():
    from paddle_amd.ops import gemm as G

    gen = torch.Generator(device="cuda").manual_seed(5)
    Bt, M, N, K = 3, 136, 264, 200
    a = torch.randn(Bt, M, K, generator=gen, device="cuda").to(torch.bfloat16)
    b = torch.randn(Bt, K, N, generator=gen, device="cuda").to(torch.bfloat16)
    c = G.gemm(a, b, M, N, K, a_kmaj=True, b_kmaj=False, batch=Bt, sA=M * K, sB=K * N)
    ref = a.float() @ b.float()
    assert (c.float() - ref).abs().max() <= 1e-2 * ref.abs().max()


def test_linear_helpers_match_torch():
    from paddle_amd.ops import gemm as G

    gen = torch.Generator(device="cuda").manual_seed(9)
    M, K, Nn = 2048, 1024, 1536
    x = torch.randn(M, K, generator=gen, device="cuda").to(torch.bfloat16)
    w = (torch.randn(K, Nn, generator=gen, device="cuda") * 0.02).to(torch.bfloat16)
    dy = torch.randn(M, Nn, generator=gen, device="cuda").to(torch.bfloat16)
    y = G.linear_fwd(x, w)
    assert torch.allclose(y.float(), x.float() @ w.float(), atol=5e-2, rtol=2e-2)
    dx = G.linear_dx(dy, w)
    assert torch.allclose(dx.float(), dy.float() @ w.float().t(), atol=5e-2, rtol=2e-2)
    mg = torch.zeros(K, Nn, device="cuda")
    G.linear_dw(x, dy, out=mg, accumulate=True)
    G.linear_dw(x, dy, out=mg, accumulate=True)
    ref = 2 * (x.float().t() @ dy.float())
    assert torch.allclose(mg, ref, atol=1e-2 * M ** 0.5, rtol=1e-4), (mg - ref).abs().max()


@pytest.mark.parametrize("M,N,K,a_kmaj,b_kmaj", [(64, 576, 100352, False, False), (128, 1152, 25000, False, False),
                                                 (256, 256, 9216, True, True)])
def test_gemm_splitk(M, N, K, a_kmaj, b_kmaj):
    from paddle_amd.ops import gemm as G

    gen = torch.Generator(device="cuda").manual_seed(3)
    a, af = _operand(M, K, a_kmaj, gen)
    b, bf = _operand(N, K, b_kmaj, gen)
    out = torch.full((M, N), 0.5, device="cuda")
    G.gemm_splitk(a, b, M, N, K, a_kmaj=a_kmaj, b_kmaj=b_kmaj, out=out, accumulate=True)
    ref = 0.5 + af @ bf.t()
    assert torch.allclose(out, ref, atol=3e-3 * K ** 0.5, rtol=1e-4), (out - ref).abs().max()


@pytest.mark.parametrize("out_f32", [True, False])
@pytest.mark.parametrize("M,N,K", [(264, 136, 72), (520, 1032, 4104)])
def test_gemm_accumulate_into_strided_output(M, N, K, out_f32):
    """C += A B^T into a column window of a wider matrix (ldc > N): the epilogue's
    per-tile C descriptor, its out-of-range lanes (rows past M, chunks past N) and
    the bf16 read-modify-write; the columns outside the window stay untouched."""
    from paddle_amd.ops import gemm as G

    gen = torch.Generator(device="cuda").manual_seed(M + N + K)
    a, af = _operand(M, K, True, gen)
    b, bf = _operand(N, K, False, gen)
    dt = torch.float32 if out_f32 else torch.bfloat16
    big = torch.randn(M, N + 40, generator=gen, device="cuda").to(dt)
    before = big.clone()
    win = big[:, 16:16 + N]
    G.gemm(a, b, M, N, K, a_kmaj=True, b_kmaj=False, out=win, accumulate=True)
    ref = before[:, 16:16 + N].float() + af @ bf.t()
    tol = (2e-3 * K ** 0.5) if out_f32 else 2e-2 * ref.abs().max().item()
    assert (big[:, 16:16 + N].float() - ref).abs().max().item() <= tol
    assert torch.equal(big[:, :16], before[:, :16]) and torch.equal(big[:, 16 + N:], before[:, 16 + N:])


@pytest.mark.parametrize("K", [64, 264, 512])
@pytest.mark.parametrize("bias", [False, True])
def test_gemm_persistent_multi_tile_direct_epilogue(K, bias):
    """More output tiles than CUs (17 x 17 = 289 > 256, ragged edges): blocks of the
    persistent grid run several tiles, so the direct-store epilogue's stores are
    still in flight while the next tile's k-tiles 0 / 1 (pre-issued) are waited on
    with the shifted counts; K = 64 has a single k-tile (k-tile 1 zero-fills)."""
    from paddle_amd.ops import gemm as G

    M = N = 4104
    gen = torch.Generator(device="cuda").manual_seed(K + bias)
    a, af = _operand(M, K, True, gen)
    b, bf = _operand(N, K, True, gen)
    bv = torch.randn(N, generator=gen, device="cuda").to(torch.bfloat16) if bias else None
    c = G.gemm(a, b, M, N, K, a_kmaj=True, b_kmaj=True, bias=bv)
    ref = af @ bf.t() + (bv.float() if bias else 0.0)
    err = (c.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item() + 1e-3, err
    # the same product twice in a row on one stream: identical bits
    c2 = G.gemm(a, b, M, N, K, a_kmaj=True, b_kmaj=True, bias=bv)
    assert torch.equal(c, c2)


@pytest.mark.parametrize("M,N,K", [(264, 136, 64), (1000, 776, 4096), (512, 1024, 8192), (4096, 512, 192)])
@pytest.mark.parametrize("a_kmaj,b_kmaj", [(True, False), (False, False), (False, True)])
@pytest.mark.parametrize("accumulate", [True, False])
def test_gemm_dw_one_wave_kernel(M, N, K, a_kmaj, b_kmaj, accumulate):
    """The one-wave-per-SIMD weight-gradient kernel (gemm1w_kernel, selected by
    pa_gemm_set_dw1w(1); off by default, measured slower): fp32 reference, ragged
    M / N edges, one and several k-tiles, and the same result as the two-wave kernel."""
    from paddle_amd.ops import _native as NL
    from paddle_amd.ops import gemm as G

    gen = torch.Generator(device="cuda").manual_seed(5)
    a, af = _operand(M, K, a_kmaj, gen)
    b, bf = _operand(N, K, b_kmaj, gen)
    c0 = torch.randn(M, N, generator=gen, device="cuda")
    outs = []
    try:
        for v in (1, 0):
            NL.lib().pa_gemm_set_dw1w(v)
            c = c0.clone() if accumulate else torch.full((M, N), float("nan"), device="cuda")
            G.gemm(a, b, M, N, K, a_kmaj=a_kmaj, b_kmaj=b_kmaj, out=c, accumulate=accumulate, alpha=0.75)
            outs.append(c)
    finally:
        NL.lib().pa_gemm_set_dw1w(0)
    ref = 0.75 * (af @ bf.t()) + (c0 if accumulate else 0)
    assert torch.allclose(outs[0], ref, atol=2e-3 * K ** 0.5, rtol=1e-4), (outs[0] - ref).abs().max()
    assert (outs[0] - outs[1]).abs().max().item() <= 1e-3 * K ** 0.5
