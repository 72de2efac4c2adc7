"""Numerics of the hand-written gfx950 kernels against plain PyTorch fp32 references.

Methodology follows the reference's OpTest (python/paddle/fluid/tests/unittests/
op_test.py:363 check_output / :395 check_grad): forward compared with a tolerance,
backward compared against an independent gradient (here autograd of the fp32
reference instead of finite differences).
"""
import math

import pytest
import torch

from paddle_amd.ops import fused as F
from paddle_amd.ops import _native

pytestmark = pytest.mark.gpu

dev = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def test_native_library_loaded():
    assert _native.available()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("H", [4096, 1000, 8192])
@pytest.mark.parametrize("with_res", [False, True])
def test_rms_norm(dtype, H, with_res):
    torch.manual_seed(0)
    Nr = 257
    x = torch.randn(Nr, H, device=dev, dtype=dtype, requires_grad=True)
    r = torch.randn(Nr, H, device=dev, dtype=dtype, requires_grad=True) if with_res else None
    w = (1 + 0.1 * torch.randn(H, device=dev, dtype=dtype)).requires_grad_()
    if with_res:
        y, h = F.rms_norm(x, w, 1e-6, residual=r)
        (y.float().pow(2).sum() + (h.float() * 0.5).sum()).backward()
    else:
        y = F.rms_norm(x, w, 1e-6)
        y.float().pow(2).sum().backward()
    xr = x.detach().float().requires_grad_()
    rr = r.detach().float().requires_grad_() if with_res else None
    wr = w.detach().float().requires_grad_()
    hr = xr + rr if with_res else xr
    yr = hr * torch.rsqrt(hr.pow(2).mean(-1, keepdim=True) + 1e-6) * wr
    loss = yr.pow(2).sum() + ((hr * 0.5).sum() if with_res else 0)
    loss.backward()
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    assert _rel(y, yr) < tol
    assert _rel(x.grad, xr.grad) < tol
    assert _rel(w.grad, wr.grad) < tol
    if with_res:
        assert _rel(r.grad, rr.grad) < tol


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_layer_norm(dtype):
    torch.manual_seed(0)
    x = torch.randn(300, 1024, device=dev, dtype=dtype, requires_grad=True)
    w = (1 + 0.1 * torch.randn(1024, device=dev, dtype=dtype)).requires_grad_()
    b = (0.1 * torch.randn(1024, device=dev, dtype=dtype)).requires_grad_()
    y = F.layer_norm(x, w, b, 1e-5)
    y.float().pow(2).sum().backward()
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = torch.nn.functional.layer_norm(xr, (1024,), wr, br, 1e-5)
    yr.pow(2).sum().backward()
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    assert _rel(y, yr) < tol
    for a, b_ in ((x, xr), (w, wr), (b, br)):
        assert _rel(a.grad, b_.grad) < tol


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("H", [5120, 8192, 4104])
def test_layer_norm_wide_rows(dtype, H):
    # 4096 < H <= 8192 takes the two-waves-per-row backward (WPR = 2); odd row count
    # leaves the last block iteration half-populated
    torch.manual_seed(0)
    Nr = 301
    x = torch.randn(Nr, H, device=dev, dtype=dtype, requires_grad=True)
    r = torch.randn(Nr, H, device=dev, dtype=dtype, requires_grad=True)
    w = (1 + 0.1 * torch.randn(H, device=dev, dtype=dtype)).requires_grad_()
    b = (0.1 * torch.randn(H, device=dev, dtype=dtype)).requires_grad_()
    y, h = F.layer_norm(x, w, b, 1e-5, residual=r)
    (y.float().pow(2).sum() + (h.float() * 0.5).sum()).backward()
    xr, rr, wr, br = (t.detach().float().requires_grad_() for t in (x, r, w, b))
    hr = xr + rr
    yr = torch.nn.functional.layer_norm(hr, (H,), wr, br, 1e-5)
    (yr.pow(2).sum() + (hr * 0.5).sum()).backward()
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    assert _rel(y, yr) < tol
    for a, b_ in ((x, xr), (r, rr), (w, wr), (b, br)):
        assert _rel(a.grad, b_.grad) < tol


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("Nr,K,M", [(2048, 512, 5120), (77, 256, 1000)])
def test_linear_bias_and_gelu(dtype, Nr, K, M):
    # bias in the GEMM epilogue; db (and dZ = dG * gelu'(Z)) from pa_bias_act_bwd
    torch.manual_seed(0)
    x = torch.randn(Nr, K, device=dev, dtype=dtype, requires_grad=True)
    w = (torch.randn(K, M, device=dev, dtype=dtype) / math.sqrt(K)).requires_grad_()
    b = torch.randn(M, device=dev, dtype=dtype).requires_grad_()
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    for fused in (F.linear, F.linear_gelu):
        for t in (x, w, b):
            t.grad = None
        y = fused(x, w, b)
        gy = torch.randn_like(y.float())
        (y.float() * gy).sum().backward()
        xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
        yr = xr @ wr + br
        if fused is F.linear_gelu:
            yr = torch.nn.functional.gelu(yr, approximate="tanh")
        (yr * gy).sum().backward()
        assert _rel(y, yr) < tol
        for a, b_ in ((x, xr), (w, wr), (b, br)):
            assert _rel(a.grad, b_.grad) < tol, fused.__name__


def test_swiglu():
    torch.manual_seed(0)
    gu = torch.randn(513, 2 * 1376, device=dev, dtype=torch.bfloat16, requires_grad=True)
    y = F.swiglu(gu)
    y.float().pow(2).sum().backward()
    gr = gu.detach().float().requires_grad_()
    g, u = gr.chunk(2, -1)
    yr = torch.nn.functional.silu(g) * u
    yr.pow(2).sum().backward()
    assert _rel(y, yr) < 1e-2
    assert _rel(gu.grad, gr.grad) < 2e-2


@pytest.mark.parametrize("V", [32000, 1001])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_softmax_ce(V, dtype):
    torch.manual_seed(0)
    x = (3 * torch.randn(129, V, device=dev)).to(dtype).requires_grad_()
    lab = torch.randint(0, V, (129,), device=dev)
    lab[5] = -100
    loss = F.softmax_cross_entropy(x, lab)
    loss.backward()
    xr = x.detach().float().requires_grad_()
    lr = torch.nn.functional.cross_entropy(xr, lab, ignore_index=-100)
    lr.backward()
    assert abs(loss.item() - lr.item()) < 1e-3 * max(1, abs(lr.item()))
    assert _rel(x.grad, xr.grad) < (2e-2 if dtype == torch.bfloat16 else 1e-4)


def test_softmax():
    torch.manual_seed(0)
    x = torch.randn(64, 777, device=dev, requires_grad=True)
    y = F.softmax(x)
    (y * torch.arange(777, device=dev)).sum().backward()
    xr = x.detach().requires_grad_()
    yr = torch.softmax(xr, -1)
    (yr * torch.arange(777, device=dev)).sum().backward()
    assert _rel(y, yr) < 1e-5
    assert _rel(x.grad, xr.grad) < 1e-4


def test_embedding():
    torch.manual_seed(0)
    W = torch.randn(1000, 256, device=dev, dtype=torch.bfloat16, requires_grad=True)
    ids = torch.randint(0, 1000, (4, 77), device=dev)
    y = F.embedding(ids, W)
    (y.float() * 2).sum().backward()
    Wr = W.detach().float().requires_grad_()
    yr = torch.nn.functional.embedding(ids, Wr)
    (yr * 2).sum().backward()
    assert _rel(y, yr) < 1e-6
    assert _rel(W.grad, Wr.grad) < 1e-2


def test_rope():
    torch.manual_seed(0)
    B, S, H, D = 2, 100, 4, 128
    cos, sin = F.rope_tables(S, D, device=dev)
    x = torch.randn(B, S, H, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    y = F.apply_rotary(x, cos, sin)
    (y.float() * torch.linspace(-1, 1, D, device=dev)).sum().backward()
    xr = x.detach().float().requires_grad_()
    yr = F._rope_ref(xr, cos, sin)
    (yr * torch.linspace(-1, 1, D, device=dev)).sum().backward()
    assert _rel(y, yr) < 1e-2
    assert _rel(x.grad, xr.grad) < 1e-2


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("S,D,Hq,Hk", [(256, 128, 4, 4), (384, 128, 4, 2), (200, 64, 2, 2), (1024, 128, 2, 2),
                                        (256, 128, 8, 2), (320, 128, 10, 2), (2048, 128, 5, 1)])
def test_flash_attention(causal, S, D, Hq, Hk):
    torch.manual_seed(0)
    B = 2
    q = torch.randn(B, S, Hq, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, Hk, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, Hk, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    do = torch.randn(B, S, Hq, D, device=dev, dtype=torch.bfloat16)
    o = F.flash_attention(q, k, v, causal=causal)
    o.backward(do)
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf = F._attn_ref(qr, kr, vr, causal, 1 / math.sqrt(D))
    orf.backward(do.float())
    assert _rel(o, orf) < 1e-2, _rel(o, orf)
    assert _rel(q.grad, qr.grad) < 2e-2, _rel(q.grad, qr.grad)
    assert _rel(k.grad, kr.grad) < 2e-2, _rel(k.grad, kr.grad)
    assert _rel(v.grad, vr.grad) < 2e-2, _rel(v.grad, vr.grad)


@pytest.mark.parametrize("S,H,Hk", [(256, 4, 4), (320, 4, 2), (1024, 8, 8), (320, 8, 2), (512, 20, 4)])
def test_rope_attention_packed(S, H, Hk):
    # D = 128 causal runs the partial-slab backward whose dQ epilogue is fused with
    # the inverse rotary (pa_fa_dq_reduce_rope) -- check the dq section separately
    torch.manual_seed(0)
    B, D = 2, 128
    cos, sin = F.rope_tables(S, D, device=dev)
    qkv = torch.randn(B, S, (H + 2 * Hk) * D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    o = F.rope_attention(qkv, cos, sin, H, Hk)
    do = torch.randn_like(o)
    o.backward(do)
    xr = qkv.detach().float().requires_grad_()
    x4 = xr.view(B, S, H + 2 * Hk, D)
    q = F._rope_ref(x4[:, :, :H], cos, sin)
    k = F._rope_ref(x4[:, :, H:H + Hk], cos, sin)
    v = x4[:, :, H + Hk:]
    k, v = k.repeat_interleave(H // Hk, 2), v.repeat_interleave(H // Hk, 2)
    orf = F._attn_ref(q, k, v, True, 1 / math.sqrt(D)).reshape(B, S, H * D)
    orf.backward(do.float())
    assert _rel(o, orf) < 1e-2
    g, gr = qkv.grad.view(B, S, -1, D), xr.grad.view(B, S, -1, D)
    assert _rel(g[:, :, :H], gr[:, :, :H]) < 2e-2, "dq"
    assert _rel(g[:, :, H:H + Hk], gr[:, :, H:H + Hk]) < 2e-2, "dk"
    assert _rel(g[:, :, H + Hk:], gr[:, :, H + Hk:]) < 2e-2, "dv"


@pytest.mark.parametrize("S,H,D,causal", [(256, 4, 128, True), (320, 2, 128, True), (256, 4, 64, True),
                                          (256, 4, 128, False)])
def test_packed_attention(S, H, D, causal):
    # GPT layout q|k|v, no rotary; causal D = 128 goes through the fused slab
    # reduce with identity cos/sin tables, the rest through the fp32 dQ accumulator
    torch.manual_seed(0)
    B = 2
    qkv = torch.randn(B, S, 3 * H * D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    o = F.packed_attention(qkv, H, causal=causal)
    do = torch.randn_like(o)
    o.backward(do)
    xr = qkv.detach().float().requires_grad_()
    x4 = xr.view(B, S, 3 * H, D)
    orf = F._attn_ref(x4[:, :, :H], x4[:, :, H:2 * H], x4[:, :, 2 * H:], causal,
                      1 / math.sqrt(D)).reshape(B, S, H * D)
    orf.backward(do.float())
    assert _rel(o, orf) < 1e-2
    g, gr = qkv.grad.view(B, S, 3, H * D), xr.grad.view(B, S, 3, H * D)
    for i, n in enumerate(("dq", "dk", "dv")):
        assert _rel(g[:, :, i], gr[:, :, i]) < 2e-2, n


def test_adamw_flat():
    from paddle_amd.ops import optim

    torch.manual_seed(0)
    n = 10007
    p = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev).to(torch.bfloat16)
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    pb = torch.empty(n, device=dev, dtype=torch.bfloat16)
    pr, mr, vr = p.clone(), m.clone(), v.clone()
    for step in range(1, 4):
        optim.adamw_flat(p, g, m, v, lr=1e-3, beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=0.1, step=step,
                         param_out=pb, decay_end=5000)
        gf = g.float()
        mr = 0.9 * mr + 0.1 * gf
        vr = 0.95 * vr + 0.05 * gf * gf
        decay = torch.where(torch.arange(n, device=dev) < 5000, 0.1, 0.0)
        pr = pr * (1 - 1e-3 * decay)
        pr = pr - 1e-3 * (mr / (1 - 0.9 ** step)) / ((vr / (1 - 0.95 ** step)).sqrt() + 1e-8)
    assert _rel(p, pr) < 1e-5
    assert _rel(pb, pr) < 1e-2


@pytest.mark.parametrize("R,C", [(64, 64), (128, 4096), (1000, 520), (16384, 4096), (72, 136)])
def test_transpose2d(R, C):
    x = torch.randn(R, C, device=dev, dtype=torch.bfloat16)
    assert torch.equal(F.transpose2d(x), x.t().contiguous())
    # strided rows (a view into a wider buffer) and batched 3-D
    big = torch.randn(R, C + 16, device=dev, dtype=torch.bfloat16)
    assert torch.equal(F.transpose2d(big[:, :C]), big[:, :C].t().contiguous())
    b = torch.randn(3, R, C, device=dev, dtype=torch.bfloat16)
    assert torch.equal(F.transpose2d(b), b.transpose(1, 2).contiguous())


def test_linear_dw_via_transpose_matches_tn():
    torch.manual_seed(0)
    T, K, Nn = 2048, 512, 768
    x = torch.randn(T, K, device=dev, dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(K, Nn, device=dev, dtype=torch.bfloat16) * 0.05).requires_grad_()
    dy = torch.randn(T, Nn, device=dev, dtype=torch.bfloat16)
    F.linear(x, w).backward(dy)
    ref = (x.detach().float().t() @ dy.float())
    assert _rel(w.grad, ref) < 1e-2
    # accumulate-into-main-grad path
    mg = torch.ones(K, Nn, device=dev, dtype=torch.bfloat16)
    w2 = w.detach().clone().requires_grad_()
    w2._pa_main_grad = mg
    F.linear(x.detach(), w2).backward(dy)
    assert _rel(mg, ref + 1) < 1e-2


def test_linear_fwd_via_transposed_weight_tracks_updates():
    torch.manual_seed(0)
    x = torch.randn(2048, 512, device=dev, dtype=torch.bfloat16)
    w = (torch.randn(512, 256, device=dev, dtype=torch.bfloat16) * 0.05).requires_grad_()
    y1 = F.linear(x, w)
    assert _rel(y1, x.float() @ w.detach().float()) < 1e-2
    with torch.no_grad():
        w.mul_(2.0)  # in-place update bumps the tensor version -> fresh W^T
    assert _rel(F.linear(x, w), x.float() @ w.detach().float()) < 1e-2
    # raw-pointer update (fused optimizer) + epoch bump
    from paddle_amd.ops import optim
    g = torch.ones_like(w)
    m, v = torch.zeros_like(w, dtype=torch.float32), torch.zeros_like(w, dtype=torch.float32)
    master = w.detach().float().clone()
    optim.adamw_flat(master.view(-1), g.view(-1), m.view(-1), v.view(-1), lr=0.1, param_out=w.data.view(-1))
    assert _rel(F.linear(x, w), x.float() @ w.detach().float()) < 1e-2


@pytest.mark.parametrize("variant", [1, 3, 4, 5])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("S,Hq,Hk", [(256, 4, 4), (384, 4, 2), (200, 2, 2), (1000, 2, 1)])
def test_flash_attention_bwd_variants(variant, causal, S, Hq, Hk):
    """Every backward kernel variant against the fp32 reference (D = 128)."""
    torch.manual_seed(1)
    B, D = 2, 128
    q = torch.randn(B, S, Hq, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, Hk, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, Hk, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    do = torch.randn(B, S, Hq, D, device=dev, dtype=torch.bfloat16)
    _native.call("pa_fa_bwd_set_variant", variant)
    split, F._FA_SPLIT = F._FA_SPLIT, False  # the single-kernel variants, not the split path
    try:
        o = F.flash_attention(q, k, v, causal=causal)
        o.backward(do)
    finally:
        _native.call("pa_fa_bwd_set_variant", 4)
        F._FA_SPLIT = split
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    F._attn_ref(qr, kr, vr, causal, 1 / math.sqrt(D)).backward(do.float())
    for a, b_ in ((q.grad, qr.grad), (k.grad, kr.grad), (v.grad, vr.grad)):
        assert _rel(a, b_) < 2e-2, _rel(a, b_)


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("Sq,Sk,Hq,Hk", [(192, 320, 4, 2), (320, 192, 2, 2), (64, 64, 2, 1), (130, 130, 3, 3),
                                          (2048, 2048, 2, 2)])
def test_flash_attention_split_bwd(causal, Sq, Sk, Hq, Hk):
    """The two-kernel backward (fa_bwd_split.hip) on ragged / unequal query and key
    lengths and GQA groups, against the fp32 reference; it must be the path taken."""
    if causal and Sq > Sk:
        pytest.skip("causal with Sq > Sk leaves query rows with no key (NaN in the reference)")
    torch.manual_seed(2)
    B, D = 2, 128
    q = torch.randn(B, Sq, Hq, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, Sk, Hk, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, Sk, Hk, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    do = torch.randn(B, Sq, Hq, D, device=dev, dtype=torch.bfloat16)
    calls = []
    orig = F._fa_bwd_split
    F._fa_bwd_split = lambda *a, **kw: calls.append(1) or orig(*a, **kw)
    try:
        o = F.flash_attention(q, k, v, causal=causal)
        o.backward(do)
    finally:
        F._fa_bwd_split = orig
    assert calls and F._FA_SPLIT
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    orf = F._attn_ref(qr, kr, vr, causal, 1 / math.sqrt(D))
    orf.backward(do.float())
    assert _rel(o, orf) < 1e-2
    for n, a, b_ in (("dq", q.grad, qr.grad), ("dk", k.grad, kr.grad), ("dv", v.grad, vr.grad)):
        assert _rel(a, b_) < 2e-2, (n, _rel(a, b_))
