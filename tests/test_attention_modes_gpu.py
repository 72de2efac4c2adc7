"""Flash-attention modes beyond the LLaMA path on the device: head dim 256, packed
variable-length batches (cu_seqlens / LoD), fp32-accumulation checks against an
fp64 reference, and the ring-attention block primitives (global-LSE backward)
in a single-process virtual ring -- each vs a plain PyTorch reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


def _ref(q, k, v, causal, scale, dtype=torch.float64):
    Hq, Hk = q.shape[2], k.shape[2]
    if Hk != Hq:
        k = k.repeat_interleave(Hq // Hk, 2)
        v = v.repeat_interleave(Hq // Hk, 2)
    qf, kf, vf = (t.to(dtype).transpose(1, 2) for t in (q, k, v))
    s = qf @ kf.transpose(-1, -2) * scale
    if causal:
        Sq, Sk = q.shape[1], k.shape[1]
        s = s.masked_fill(~torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).tril(Sk - Sq), float("-inf"))
    return (torch.softmax(s, -1) @ vf).transpose(1, 2)


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).abs().max() / b.abs().max()).item()


@pytest.mark.parametrize("D,causal", [(256, True), (256, False), (128, True), (64, False)])
def test_flash_attention_head_dims(D, causal):
    from paddle_amd import ops

    g = torch.Generator(device=dev).manual_seed(D)
    B, S, H = 2, 384, 4
    q, k, v = (torch.randn(B, S, H, D, generator=g, device=dev).to(torch.bfloat16).requires_grad_() for _ in range(3))
    o = ops.flash_attention(q, k, v, causal=causal)
    qr, kr, vr = (t.detach().double().requires_grad_() for t in (q, k, v))
    orf = _ref(qr, kr, vr, causal, D ** -0.5)
    assert _rel(o, orf) < 1e-2  # bf16 output rounding; fp32 accumulation inside
    do = torch.randn(o.shape, generator=g, device=dev).to(torch.bfloat16)
    o.backward(do)
    orf.backward(do.double())
    for a, b in ((q, qr), (k, kr), (v, vr)):
        assert _rel(a.grad, b.grad) < 3e-2


@pytest.mark.parametrize("causal,hk", [(True, 4), (False, 4), (True, 2)])
def test_flash_attention_varlen(causal, hk):
    from paddle_amd import ops

    g = torch.Generator(device=dev).manual_seed(3)
    lens = [130, 0, 64, 257, 1]
    cu = [0]
    for n in lens:
        cu.append(cu[-1] + n)
    T, H, D = cu[-1], 4, 128
    q = torch.randn(T, H, D, generator=g, device=dev).to(torch.bfloat16).requires_grad_()
    k, v = (torch.randn(T, hk, D, generator=g, device=dev).to(torch.bfloat16).requires_grad_() for _ in range(2))
    o = ops.flash_attention_varlen(q, k, v, cu, causal=causal)
    do = torch.randn(o.shape, generator=g, device=dev).to(torch.bfloat16)
    o.backward(do)
    qr, kr, vr = (t.detach().double().requires_grad_() for t in (q, k, v))
    parts = []
    for i in range(len(lens)):
        a, b = cu[i], cu[i + 1]
        if b > a:
            parts.append(_ref(qr[a:b][None], kr[a:b][None], vr[a:b][None], causal, D ** -0.5)[0])
    orf = torch.cat(parts)
    orf.backward(do.double())
    assert _rel(o, orf) < 1e-2
    for a, b in ((q, qr), (k, kr), (v, vr)):
        assert _rel(a.grad, b.grad) < 3e-2


def test_ring_attention_blocks_virtual_ring():
    """The per-rank schedule of ring_attention (zigzag pairs, LSE merge, global-LSE
    backward) on the device kernels, every rank simulated in one process."""
    from paddle_amd.distributed.fleet import context_parallel as cp

    P, B, H, D = 4, 1, 4, 128
    S = 2 * P * 128
    g = torch.Generator(device=dev).manual_seed(9)
    q, k, v = (torch.randn(B, S, H, D, generator=g, device=dev).to(torch.bfloat16) for _ in range(3))
    scale = D ** -0.5
    shards = [[cp.zigzag_split(t, r, P) for t in (q, k, v)] for r in range(P)]
    c = S // (2 * P)
    outs, lses = [], []
    for r in range(P):
        qh = (shards[r][0][:, :c], shards[r][0][:, c:])
        acc = [[None, None], [None, None]]
        for src in range(P):
            kk, vv = shards[src][1], shards[src][2]
            for a, b, causal in cp._pairs(r, src, P):
                o, lse = cp._block_fwd(qh[a], kk[:, b * c:(b + 1) * c], vv[:, b * c:(b + 1) * c], causal, scale)
                acc[a][0], acc[a][1] = cp._merge(acc[a][0], acc[a][1], o, lse)
        outs.append(torch.cat([acc[0][0], acc[1][0]], 1))
        lses.append(torch.cat([acc[0][1], acc[1][1]], 2))
    o_full = cp.zigzag_merge(outs)
    ref = _ref(q, k, v, True, scale)
    assert _rel(o_full, ref) < 1e-2
    # backward of one (q half, kv half) pair with the global LSE equals the slice of the full gradient
    qr, kr, vr = (t.double().requires_grad_() for t in (q, k, v))
    orf = _ref(qr, kr, vr, True, scale)
    do = torch.randn(orf.shape, generator=g, device=dev)
    orf.backward(do)
    r = 1
    o_r = outs[r].to(torch.bfloat16)
    do_r = cp.zigzag_split(do.to(torch.bfloat16), r, P)
    dq = torch.zeros(B, 2 * c, H, D, device=dev)
    for src in range(P):
        kk, vv = shards[src][1], shards[src][2]
        for a, b, causal in cp._pairs(r, src, P):
            gq, _, _ = cp._block_bwd(shards[r][0][:, a * c:(a + 1) * c], kk[:, b * c:(b + 1) * c],
                                     vv[:, b * c:(b + 1) * c], o_r[:, a * c:(a + 1) * c],
                                     do_r[:, a * c:(a + 1) * c], lses[r][:, :, a * c:(a + 1) * c].contiguous(),
                                     causal, scale)
            dq[:, a * c:(a + 1) * c] += gq
    assert _rel(dq, cp.zigzag_split(qr.grad, r, P)) < 3e-2
