"""Split-K for under-filled GEMMs (ops/gemm.py split_k_for: 320 tiles on 256 CUs):
k-slices into fp32 slabs + the deterministic summing pass (pa_gemm_splitk_sum, bias
folded in) match the fp32 product, for the K-major and MN-major B forms."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("b_kmaj", [True, False])
@pytest.mark.parametrize("with_bias", [False, True])
def test_splitk_gemm_matches_fp32(b_kmaj, with_bias):
    from paddle_amd.ops import gemm as G

    M, N, K = 4096, 5120, 20480
    assert G.split_k_for(M, N, K) > 1
    g = torch.Generator(device="cuda").manual_seed(1)
    a = (torch.randn(M, K, generator=g, device="cuda") / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, K, generator=g, device="cuda").to(torch.bfloat16)
    bm = b if b_kmaj else b.t().contiguous()
    bias = torch.randn(N, device="cuda").to(torch.bfloat16) if with_bias else None
    out = G.gemm(a, bm, M, N, K, a_kmaj=True, b_kmaj=b_kmaj, bias=bias)
    ref = a.float() @ b.float().t() + (bias.float() if with_bias else 0)
    err = (out.float() - ref).abs().max() / ref.abs().max()
    assert err < 1e-2, float(err)
    # deterministic: the same bits twice
    assert torch.equal(out, G.gemm(a, bm, M, N, K, a_kmaj=True, b_kmaj=b_kmaj, bias=bias))


def test_full_grids_do_not_split():
    from paddle_amd.ops import gemm as G

    assert G.split_k_for(16384, 4096, 4096) == 1
    assert G.split_k_for(4096, 5120, 5120) == 1  # slab traffic would cost more than the idle CUs
