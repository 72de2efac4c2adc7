"""Fused GEMM epilogues (csrc/kernels/gemm.hip EPI 1-3, ops.gemm.gemm_epi) and the
model nodes built on them (ops.swiglu_mlp, ops.qkv_rope_attention), against the
unfused kernels / fp32 torch references."""
import math

import pytest
import torch

from paddle_amd import ops
from paddle_amd.ops import fused as F
from paddle_amd.ops import gemm as G

pytestmark = pytest.mark.gpu
dev = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def _bf(*shape, s=1.0):
    return (torch.randn(*shape, device=dev) * s).to(torch.bfloat16)


def test_epi_swiglu_forward():
    torch.manual_seed(0)
    T, K, N2 = 1536, 512, 1280  # partial last tile rows / columns
    x, w = _bf(T, K), _bf(K, N2, s=0.05)
    wt = F.transpose2d(w)
    gu = torch.empty(T, N2, device=dev, dtype=torch.bfloat16)
    h = torch.empty(T, N2 // 2, device=dev, dtype=torch.bfloat16)
    G.gemm_epi(G.EPI_SWIGLU_FWD, x, wt, T, N2, K, out=gu, aux=h)
    plain = G.gemm(x, wt, T, N2, K, a_kmaj=True, b_kmaj=True)
    assert torch.equal(gu, plain)  # same main loop, same rounding
    g, u = ops.deinterleave_gate_up(gu.float())
    ref = torch.nn.functional.silu(g) * u
    assert _rel(h, ref) < 1e-2


def test_epi_swiglu_backward():
    torch.manual_seed(1)
    T, H, I = 1280, 512, 640
    dy, wd = _bf(T, H), _bf(I, H, s=0.05)
    gu = _bf(T, 2 * I)
    dgu = torch.empty(T, 2 * I, device=dev, dtype=torch.bfloat16)
    G.gemm_epi(G.EPI_SWIGLU_BWD, dy, wd, T, I, H, out=dgu, aux=gu)
    da = (dy.float() @ wd.float().t()).to(torch.bfloat16).float()
    g, u = ops.deinterleave_gate_up(gu.float())
    sg = torch.sigmoid(g)
    ref = ops.interleave_gate_up(da * u * sg * (1 + g * (1 - sg)), da * g * sg)
    assert _rel(dgu, ref) < 1.5e-2


@pytest.mark.parametrize("S", [512, 2048])
def test_epi_rope_matches_gemm_plus_rope(S):
    torch.manual_seed(2)
    B, K, Hq, Hk, D = 2, 512, 4, 2, 128
    W = (Hq + 2 * Hk) * D
    T = B * S
    y, w = _bf(T, K), _bf(K, W, s=0.05)
    wt = F.transpose2d(w)
    cos, sin = ops.rope_tables(4096, D, 500000.0, device=dev)
    out = torch.empty(T, W, device=dev, dtype=torch.bfloat16)
    G.gemm_epi(G.EPI_ROPE, y, wt, T, W, K, out=out, cos=cos, sin=sin, rope_cols=(Hq + Hk) * D, rope_S=S)
    qkv = G.gemm(y, wt, T, W, K, a_kmaj=True, b_kmaj=True).view(B, S, Hq + 2 * Hk, D)
    ref = torch.cat([F._rope_ref(qkv[:, :, :Hq + Hk], cos, sin), qkv[:, :, Hq + Hk:]], 2).reshape(T, W)
    v0 = (Hq + Hk) * D
    assert torch.equal(out[:, v0:], ref[:, v0:])  # v columns pass through
    assert _rel(out[:, :v0], ref[:, :v0]) < 1e-2


def _grads(fn, *ts):
    ts = [t.detach().clone().requires_grad_(True) for t in ts]
    out = fn(*ts)
    g = torch.randn_like(out)
    out.backward(g)
    return out.detach(), [t.grad for t in ts]


def test_swiglu_mlp_fused_matches_unfused(monkeypatch):
    torch.manual_seed(3)
    B, S, H, I = 1, 2048, 512, 1024
    x = _bf(B, S, H)
    wgu = torch.nn.Parameter(_bf(H, 2 * I, s=0.05))
    wd = torch.nn.Parameter(_bf(I, H, s=0.05))
    assert F.swiglu_mlp_fused_ok(x, wgu, wd)
    torch.manual_seed(9)
    y1, g1 = _grads(ops.swiglu_mlp, x, wgu, wd)
    monkeypatch.setattr(F, "swiglu_mlp_fused_ok", lambda *a: False)
    torch.manual_seed(9)
    y2, g2 = _grads(ops.swiglu_mlp, x, wgu, wd)
    assert _rel(y1, y2) < 1e-2
    for a, b in zip(g1, g2):
        assert _rel(a, b) < 2e-2


def test_qkv_rope_attention_fused_matches_unfused(monkeypatch):
    torch.manual_seed(4)
    B, S, H, Hq, Hk, D = 1, 2048, 512, 4, 2, 128
    y = _bf(B, S, H)
    w = torch.nn.Parameter(_bf(H, (Hq + 2 * Hk) * D, s=0.05))
    cos, sin = ops.rope_tables(4096, D, 500000.0, device=dev)
    assert F._qkv_rope_fused_ok(y, w, cos, Hq, Hk)
    f = lambda a, b: ops.qkv_rope_attention(a, b, cos, sin, Hq, Hk)
    torch.manual_seed(9)
    o1, g1 = _grads(f, y, w)
    monkeypatch.setattr(F, "_qkv_rope_fused_ok", lambda *a: False)
    torch.manual_seed(9)
    o2, g2 = _grads(f, y, w)
    assert _rel(o1, o2) < 1e-2
    for a, b in zip(g1, g2):
        assert _rel(a, b) < 2e-2


def test_llama_block_uses_fused_nodes(monkeypatch):
    """The LLaMA decoder runs the fused nodes (and their launches) on the GPU."""
    from paddle_amd.models.llama import LLAMA_CONFIGS, LlamaConfig, LlamaForCausalLM

    cfg = LlamaConfig(**dict(LLAMA_CONFIGS["llama-tiny"], hidden_size=512, intermediate_size=1024,
                             num_attention_heads=4, max_position_embeddings=2048))
    m = LlamaForCausalLM(cfg, dev)
    calls = []
    orig = G.gemm_epi
    monkeypatch.setattr(G, "gemm_epi", lambda epi, *a, **k: calls.append(epi) or orig(epi, *a, **k))
    ids = torch.randint(0, cfg.vocab_size, (1, 2049), device=dev)
    loss = m(ids[:, :-1], ids[:, 1:])
    loss.backward()
    L = cfg.num_hidden_layers
    assert calls.count(G.EPI_ROPE) == L and calls.count(G.EPI_SWIGLU_FWD) == L and calls.count(G.EPI_SWIGLU_BWD) == L
    assert math.isfinite(loss.item())
