"""fp8 (OCP e4m3) quantisation kernels and the block-scaled MFMA GEMM (gemm.hip
pa_gemm_f8) against fp32 references of the same quantised operands."""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"
F8 = torch.float8_e4m3fn


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def test_quant_rows_matches_torch_e4m3():
    from paddle_amd.ops import fp8

    g = torch.Generator(device=dev).manual_seed(0)
    x = (torch.randn(64, 1024, generator=g, device=dev) * torch.logspace(-3, 3, 64, device=dev)[:, None])
    x = x.to(torch.bfloat16)
    q, s = fp8.quant_rows(x)
    amax = x.float().abs().amax(1)
    assert torch.allclose(s, amax / 448, rtol=1e-6)
    ref = (x.float().cpu() / s.cpu()[:, None]).clamp(-448, 448).to(F8)
    same = (q.cpu().view(torch.uint8) == ref.view(torch.uint8)).float().mean().item()
    assert same > 0.999, same  # x * (1/s) vs x / s may round differently in the last bit
    deq = q.float() * s[:, None]
    # relative 2^-4 for normals; absolute half a subnormal step (2^-10 * scale) below 2^-6 * scale
    assert ((deq - x.float()).abs() <= 0.0625 * x.float().abs() + s[:, None] * 2.0 ** -9).all()


def test_quant_cols_t():
    from paddle_amd.ops import fp8

    g = torch.Generator(device=dev).manual_seed(1)
    w = torch.randn(3, 160, 200, generator=g, device=dev).to(torch.bfloat16)
    qt, s = fp8.quant_cols_t(w)
    assert qt.shape == (3, 200, 160) and s.shape == (3, 200)
    assert torch.allclose(s, w.float().abs().amax(1) / 448, rtol=1e-6)
    deq = qt.float() * s[:, :, None]
    assert _rel(deq, w.float().transpose(1, 2)) < 0.07


@pytest.mark.parametrize("M,N,K", [(256, 256, 256), (300, 520, 784), (1024, 768, 4096)])
def test_gemm_f8_exact_on_quantised_operands(M, N, K):
    from paddle_amd.ops import fp8

    g = torch.Generator(device=dev).manual_seed(M + N + K)
    a = torch.randn(M, K, generator=g, device=dev).to(torch.bfloat16)
    b = torch.randn(N, K, generator=g, device=dev).to(torch.bfloat16)
    aq, sa = fp8.quant_rows(a)
    bq, sb = fp8.quant_rows(b)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    fp8.gemm_f8(aq, sa, bq, sb, M, N, K, out=out)
    ref = (aq.float() * sa[:, None]) @ (bq.float() * sb[:, None]).t()
    assert _rel(out, ref) < 1e-2
    # and against the unquantised product: e4m3 error only
    assert _rel(out, a.float() @ b.float().t()) < 0.1


def test_grouped_swiglu_fp8_close_to_bf16():
    from paddle_amd.ops import grouped

    counts = [0, 5, 300, 1, 64, 777, 33, 0]
    g = torch.Generator(device=dev).manual_seed(3)
    H, I, R, E = 256, 128, sum(counts), len(counts)
    x = torch.randn(R, H, generator=g, device=dev).to(torch.bfloat16)
    gu = (torch.randn(E, H, 2 * I, generator=g, device=dev) / H ** 0.5).to(torch.bfloat16)
    dn = (torch.randn(E, I, H, generator=g, device=dev) / I ** 0.5).to(torch.bfloat16)
    dy = torch.randn(R, H, generator=g, device=dev).to(torch.bfloat16)
    res = []
    for f8 in (False, True):
        xx, gg, dd = (t.clone().requires_grad_() for t in (x, gu, dn))
        y = grouped.grouped_swiglu_mlp(xx, gg, dd, counts, fp8=f8)
        y.backward(dy)
        res.append((y, xx.grad, gg.grad, dd.grad))
    for a, b in zip(*res):
        assert _rel(b, a) < 0.12
        cos = torch.nn.functional.cosine_similarity(a.float().flatten(), b.float().flatten(), dim=0).item()
        assert cos > 0.995, cos
