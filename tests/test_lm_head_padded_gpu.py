"""Tied LM head with a vocabulary that is not a multiple of 8 (GPT's 50,257) on the
hand-written GEMM: ``pa_gemm_padded`` runs the forward, dX and dW forms on 8-aligned
row buffers (no hipBLASLt / ATen product left in the head)."""
import pytest
import torch

from paddle_amd.autograd import tape
from paddle_amd.ops import fused as F
from paddle_amd.ops import gemm as G
from paddle_amd.utils import strict

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


@pytest.mark.parametrize("V", [1003, 50257])
@pytest.mark.parametrize("main_grad", [False, True])
def test_tied_head_ragged_vocab_matches_fp32(V, main_grad, monkeypatch):
    torch.manual_seed(0)
    T, H = 1024, 256
    x = (torch.randn(T, H, device="cuda") * 0.5).to(torch.bfloat16)
    w = torch.nn.Parameter((torch.randn(V, H, device="cuda") * 0.05).to(torch.bfloat16))
    if main_grad:
        w._pa_main_grad = torch.zeros(V, H, device="cuda")
        w._pa_grad_fresh = True
    dy = torch.randn(T, V, device="cuda").to(torch.bfloat16)
    calls = []
    orig = G.gemm_padded
    monkeypatch.setattr(G, "gemm_padded", lambda *a, **k: calls.append(1) or orig(*a, **k))
    xx = x.clone()
    with strict.region("lm_head:test"):
        with tape.recording() as t:
            t.watch(xx)
            y = F.linear_t(xx, w)
        t.backward(y, dy)
    gx = t.grad(xx)
    gw = w._pa_main_grad if main_grad else w.grad
    ref_y = x.float() @ w.float().t()
    assert _rel(y, ref_y) < 1e-2
    assert _rel(gx, dy.float() @ w.float()) < 1e-2
    assert _rel(gw, dy.float().t() @ x.float()) < 1e-2
    assert len(calls) == 3  # forward, dX, dW all on the padded MFMA GEMM


def test_padded_gemm_contract_rejects_unaligned_rows():
    a = torch.zeros(64, 250, device="cuda", dtype=torch.bfloat16)[:, :250]  # ld 250: not 8-aligned
    b = torch.zeros(16, 250, device="cuda", dtype=torch.bfloat16)
    out = torch.empty(64, 16, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        G.gemm_padded(a, b, 64, 16, 250, a_kmaj=True, b_kmaj=True, out=out)
