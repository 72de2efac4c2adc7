"""Ragged grouped GEMM (ops/grouped.py, gemm.hip grp_mode 1/2) against per-group
fp32 references, and the grouped-expert ERNIE-MoE path against the per-expert loop
over several optimizer steps (the configuration that faulted in round 1,
profiles/r1_moe_grouped_probe.md)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"

# ragged: empty groups, sizes not a multiple of 8 or of the 256-row tile, one > 2 tiles
COUNTS = [0, 5, 300, 1, 0, 64, 777, 33]


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def _offs(counts):
    o = [0]
    for c in counts:
        o.append(o[-1] + c)
    return o


# > 64 groups: the device-side tile schedule scans the offsets in chunks of 64
MANY = [(7 * i) % 23 * (i % 3 != 0) for i in range(130)]


@pytest.mark.parametrize("b_kmaj,counts", [(False, COUNTS), (True, COUNTS), (False, MANY)])
def test_grouped_rows(b_kmaj, counts):
    from paddle_amd.ops import gemm as G

    g = torch.Generator(device=dev).manual_seed(int(b_kmaj))
    K, Nn, R = 192, 320, sum(counts)
    o = _offs(counts)
    a = torch.randn(R, K, generator=g, device=dev).to(torch.bfloat16)
    shape = (len(counts), Nn, K) if b_kmaj else (len(counts), K, Nn)
    b = (torch.randn(*shape, generator=g, device=dev) / K ** 0.5).to(torch.bfloat16)
    out = torch.full((R, Nn), float("nan"), device=dev).to(torch.bfloat16)
    G.grouped_rows(a, b, G.group_table(torch.tensor(o, dtype=torch.int32, device=dev), R), b_kmaj=b_kmaj, out=out)
    for e in range(len(counts)):
        w = b[e].float().t() if b_kmaj else b[e].float()
        ref = a[o[e]:o[e + 1]].float() @ w
        if counts[e]:
            assert _rel(out[o[e]:o[e + 1]], ref) < 1e-2, e


@pytest.mark.parametrize("accumulate", [False, True])
def test_grouped_dw(accumulate):
    from paddle_amd.ops import gemm as G

    g = torch.Generator(device=dev).manual_seed(7)
    M, Nn, R = 136, 264, sum(COUNTS)
    o = _offs(COUNTS)
    a = torch.randn(R, M, generator=g, device=dev).to(torch.bfloat16)
    b = torch.randn(R, Nn, generator=g, device=dev).to(torch.bfloat16)
    init = torch.randn(len(COUNTS), M, Nn, generator=g, device=dev)
    out = init.clone()
    G.grouped_dw(a, b, torch.tensor(o, dtype=torch.int32, device=dev), out, accumulate=accumulate)
    for e in range(len(COUNTS)):
        ref = a[o[e]:o[e + 1]].float().t() @ b[o[e]:o[e + 1]].float()
        if accumulate:
            ref = ref + init[e]
        assert (out[e] - ref).abs().max().item() <= 2e-3 * max(ref.abs().max().item(), 1.0), e


def test_grouped_swiglu_mlp_fwd_bwd():
    from paddle_amd.ops import grouped

    g = torch.Generator(device=dev).manual_seed(3)
    H, I, R = 256, 128, sum(COUNTS)
    E = len(COUNTS)
    x = torch.randn(R, H, generator=g, device=dev).to(torch.bfloat16).requires_grad_()
    gu = (torch.randn(E, H, 2 * I, generator=g, device=dev) / H ** 0.5).to(torch.bfloat16).requires_grad_()
    dn = (torch.randn(E, I, H, generator=g, device=dev) / I ** 0.5).to(torch.bfloat16).requires_grad_()
    assert grouped.supported(x, gu, dn)
    y = grouped.grouped_swiglu_mlp(x, gu, dn, COUNTS)
    dy = torch.randn(R, H, generator=g, device=dev).to(torch.bfloat16)
    y.backward(dy)
    xr, gur, dnr = (t.detach().float().requires_grad_() for t in (x, gu, dn))
    o = _offs(COUNTS)
    parts = []
    for e in range(E):
        h = xr[o[e]:o[e + 1]] @ gur[e]
        gt, up = h.chunk(2, -1)
        parts.append((torch.nn.functional.silu(gt) * up) @ dnr[e])
    yr = torch.cat(parts)
    yr.backward(dy.float())
    assert _rel(y, yr) < 2e-2
    assert _rel(x.grad, xr.grad) < 3e-2
    assert _rel(gu.grad, gur.grad) < 3e-2
    assert _rel(dn.grad, dnr.grad) < 3e-2


def test_ernie_moe_grouped_matches_loop_over_steps():
    """ernie-moe-tiny (widened to MFMA-sized experts) trained 4 steps with the
    sharded optimizer's fp32 main_grad, grouped vs per-expert: losses agree."""
    from paddle_amd.models.ernie_moe import ERNIE_MOE_CONFIGS, ErnieMoEConfig, ErnieMoEForCausalLM
    from paddle_amd.parallel.sharding import FlatShardedOptimizer

    kw = dict(ERNIE_MOE_CONFIGS["ernie-moe-tiny"])
    kw.update(hidden_size=256, moe_intermediate_size=128, num_experts=8, top_k=2)
    ids = torch.randint(0, kw["vocab_size"], (4, 129), generator=torch.Generator().manual_seed(5)).to(dev)
    curves = []
    for grouped in (False, True):
        torch.manual_seed(0)
        m = ErnieMoEForCausalLM(ErnieMoEConfig(**kw, grouped_experts=grouped), dev)
        assert m.layers[1].moe.grouped == grouped
        opt = FlatShardedOptimizer(m.named_parameters(), lr=1e-3)
        losses = []
        for _ in range(4):
            loss = m(ids[:, :-1], ids[:, 1:])
            loss.backward()
            opt.step()
            opt.zero_grad()
            losses.append(loss.item())
        torch.cuda.synchronize()
        curves.append(losses)
    print(curves)
    for a, b in zip(*curves):
        assert abs(a - b) < 2e-2 * max(abs(a), 1.0), curves
    assert curves[1][-1] < curves[1][0]


def test_moe_dispatch_combine_kernels():
    """Native dispatch / combine (and their backward gathers) vs the torch indexing
    path, with dropped slots (capacity) in the routing."""
    from paddle_amd.ops import moe_route as R

    g = torch.Generator(device=dev).manual_seed(11)
    T, k, E, H = 300, 3, 8, 264
    flat_e = torch.randint(0, E, (T * k,), generator=g, device=dev)
    keep = torch.rand(T * k, generator=g, device=dev) > 0.2
    _, src, pos, _ = R.routing(flat_e, T, k, keep)
    x = torch.randn(T, H, generator=g, device=dev).to(torch.bfloat16)
    w = torch.rand(T * k, generator=g, device=dev)
    dy = torch.randn(T, H, generator=g, device=dev).to(torch.bfloat16)
    outs = []
    for native in (True, False):
        xx = x.clone().requires_grad_()
        ww = w.clone().requires_grad_()
        if native:
            send = R.dispatch(xx, src, pos, k)
            y = R.combine(send * 2, ww, pos, k)
        else:
            send = xx[src.long()]
            keep_s = (pos >= 0).nonzero().squeeze(-1)
            y = torch.zeros(T, H, device=dev).index_add(
                0, keep_s // k, (send.float() * 2)[pos[keep_s].long()] * ww[keep_s].unsqueeze(-1))
        y.backward(dy)
        outs.append((y.float(), xx.grad.float(), ww.grad.float()))
    for a, b in zip(*outs):
        assert _rel(a, b) < 1e-2
    assert (outs[0][2][~keep] == 0).all()


def test_moe_capacity_sync_free_layer_matches_exact_split():
    """Fixed-capacity MoE layer (padded [expert, capacity] slabs, grouped experts on
    the padded rows, combine with zero gradient for padding rows) vs the exact-split
    path with the same capacity on the device: outputs and input / expert / gate
    gradients agree."""
    from paddle_amd.distributed.fleet import MoELayer, TopKGate
    from paddle_amd.models.ernie_moe import ERNIE_MOE_CONFIGS, ErnieMoEConfig, ErnieMoEForCausalLM

    kw = dict(ERNIE_MOE_CONFIGS["ernie-moe-tiny"])
    kw.update(hidden_size=256, moe_intermediate_size=128, num_experts=8, top_k=2)
    torch.manual_seed(0)
    m = ErnieMoEForCausalLM(ErnieMoEConfig(**kw, grouped_experts=True), dev)
    experts = m.layers[1].moe.experts
    gate = TopKGate(256, 8, top_k=2, capacity_factor=0.75)
    gate.weight.data = (torch.randn(256, 8, generator=torch.Generator().manual_seed(3)) * 0.3).to(dev)
    x0 = torch.randn(384, 256, generator=torch.Generator().manual_seed(4)).to(dev).to(torch.bfloat16)
    dy = torch.randn(384, 256, generator=torch.Generator().manual_seed(6)).to(dev).to(torch.bfloat16)
    res = []
    for sf in (True, False):
        layer = MoELayer(256, experts, gate=gate, capacity_factor=0.75, sync_free=sf)
        for p in list(experts.parameters()) + [gate.weight]:
            p.grad = None
        x = x0.clone().requires_grad_()
        y = layer(x)
        y.backward(dy)
        res.append((y.float(), x.grad.float(), [p.grad.float().clone() for p in experts.parameters()],
                    gate.weight.grad.float().clone()))
    (ya, xa, pa, ga), (yb, xb, pb, gb) = res
    assert _rel(ya, yb) < 1e-2 and _rel(xa, xb) < 2e-2 and _rel(ga, gb) < 2e-2
    for a, b in zip(pa, pb):
        assert _rel(a, b) < 2e-2


@pytest.mark.parametrize("fp8", [False, True])
@pytest.mark.parametrize("accumulate", [False, True])
@pytest.mark.parametrize("nmb", [1, 3])
def test_grouped_dw_images(fp8, accumulate, nmb):
    """Expert dW over the K-major token images (fp8.hip pa_group_image: expert rows of
    several micro-batches concatenated per expert into 64-aligned segments, bf16 or
    e4m3 with per-(expert, channel) scales) and the grouped-K GEMM, against the fp32
    sum over micro-batches of the per-expert products; experts without tokens get 0."""
    from paddle_amd.ops import grouped as GR
    from paddle_amd.ops import gemm as G

    g = torch.Generator(device=dev).manual_seed(11 + nmb)
    M, Nn = 192, 320
    E = len(COUNTS)
    mbs = []
    for j in range(nmb):
        counts = COUNTS if j % 2 == 0 else MANY[:E]
        R = sum(counts)
        a = torch.randn(R, M, generator=g, device=dev).to(torch.bfloat16)
        b = (torch.randn(R, Nn, generator=g, device=dev) * 1e-3).to(torch.bfloat16)  # gradient-sized
        o = _offs(counts)
        mbs.append((a, b, o, G.group_table(torch.tensor(o, dtype=torch.int32, device=dev), R), counts))
    cum, poffs = GR._cat_offsets([m[3] for m in mbs], E)
    tot = [sum(m[4][e] for m in mbs) for e in range(E)]
    pl = poffs.cpu().tolist()
    assert all(p % 64 == 0 for p in pl) and all(pl[e + 1] - pl[e] == (c + 63) // 64 * 64 for e, c in enumerate(tot))
    w = torch.zeros(E, M, Nn, device=dev)
    init = torch.randn(E, M, Nn, generator=g, device=dev) * 1e-3
    if accumulate:
        w._pa_main_grad = init.clone()
        w._pa_grad_fresh = False
        assert GR._wgrad_images(w, [m[0] for m in mbs], [m[1] for m in mbs], [m[3] for m in mbs], E, fp8) is None
        got = w._pa_main_grad
    else:
        got = GR._wgrad_images(w, [m[0] for m in mbs], [m[1] for m in mbs], [m[3] for m in mbs], E, fp8)
    tol = 6e-2 if fp8 else 1e-2
    for e in range(E):
        ref = sum(m[0][m[2][e]:m[2][e + 1]].float().t() @ m[1][m[2][e]:m[2][e + 1]].float() for m in mbs)
        base = init[e] if accumulate else torch.zeros(M, Nn, device=dev)
        d = got[e] - base
        if tot[e] == 0:
            assert not torch.any(d), e
            continue
        err = (d - ref).norm() / ref.norm().clamp_min(1e-30)
        assert err < tol, (e, tot[e], float(err))


def test_ernie_moe_deferred_expert_dw_matches_per_microbatch():
    """accum.deferring() (the optimizer's no_sync): the expert dW of the first
    micro-batches is computed with the last one in one grouped GEMM; the main_grad
    after the step equals the per-micro-batch accumulation."""
    from paddle_amd.autograd import tape
    from paddle_amd.models.ernie_moe import ERNIE_MOE_CONFIGS, ErnieMoEConfig, ErnieMoEForCausalLM
    from paddle_amd.ops import accum, grouped as GR
    from paddle_amd.parallel.sharding import FlatShardedOptimizer

    def grads(defer):
        torch.manual_seed(0)
        cfg = ErnieMoEConfig(**dict(ERNIE_MOE_CONFIGS["ernie-moe-tiny"], hidden_size=256, moe_intermediate_size=128,
                                    intermediate_size=512, grouped_experts=True, max_position_embeddings=512,
                                    num_experts=8))
        m = ErnieMoEForCausalLM(cfg, torch.device(dev))
        opt = FlatShardedOptimizer(m.named_parameters(), lr=0.0, grad_dtype=torch.float32)
        gen = torch.Generator().manual_seed(5)
        for j in range(3):
            ids = torch.randint(0, cfg.vocab_size, (2, 257), generator=gen).to(dev)
            ctx = opt.no_sync() if (defer and j < 2) else __import__("contextlib").nullcontext()
            with ctx:
                with tape.recording() as t:
                    loss = m(ids[:, :-1], ids[:, 1:])
                t.backward(loss)
        assert not GR._STASH
        torch.cuda.synchronize()
        return {n: p._pa_main_grad.clone() for n, p in m.named_parameters() if "gate_up" in n or "down" in n}

    old = GR._DEFER_ON
    try:
        GR._DEFER_ON = False
        ref = grads(False)
        GR._DEFER_ON = True
        got = grads(True)
    finally:
        GR._DEFER_ON = old
        accum.set_deferring(False)
    assert ref.keys() == got.keys() and ref
    for n in ref:
        err = (got[n] - ref[n]).norm() / ref[n].norm().clamp_min(1e-30)
        assert err < 1e-2, (n, float(err))


def test_abandoned_accumulation_does_not_leak_deferred_expert_dw():
    """no_sync micro-batches followed by zero_grad WITHOUT a step (an AMP
    inf skip, a discarded batch) must not leave their deferred expert-dW operands in
    the stash: the next step's main_grad equals the non-deferred path's."""
    from paddle_amd.autograd import tape
    from paddle_amd.models.ernie_moe import ERNIE_MOE_CONFIGS, ErnieMoEConfig, ErnieMoEForCausalLM
    from paddle_amd.ops import accum, grouped as GR
    from paddle_amd.parallel.sharding import FlatShardedOptimizer

    def grads(defer):
        torch.manual_seed(0)
        cfg = ErnieMoEConfig(**dict(ERNIE_MOE_CONFIGS["ernie-moe-tiny"], hidden_size=256, moe_intermediate_size=128,
                                    intermediate_size=512, grouped_experts=True, max_position_embeddings=512,
                                    num_experts=8))
        m = ErnieMoEForCausalLM(cfg, torch.device(dev))
        opt = FlatShardedOptimizer(m.named_parameters(), lr=0.0, grad_dtype=torch.float32)
        gen = torch.Generator().manual_seed(6)
        batches = [torch.randint(0, cfg.vocab_size, (2, 257), generator=gen).to(dev) for _ in range(3)]
        # abandoned accumulation: one no_sync micro-batch, then zero_grad with no step
        with opt.no_sync():
            with tape.recording() as t:
                loss = m(batches[0][:, :-1], batches[0][:, 1:])
            t.backward(loss)
        opt.zero_grad()
        assert not GR._STASH
        for j in (1, 2):
            ctx = opt.no_sync() if (defer and j == 1) else __import__("contextlib").nullcontext()
            with ctx:
                with tape.recording() as t:
                    loss = m(batches[j][:, :-1], batches[j][:, 1:])
                t.backward(loss)
        torch.cuda.synchronize()
        return {n: p._pa_main_grad.clone() for n, p in m.named_parameters() if "gate_up" in n or "down" in n}

    old = GR._DEFER_ON
    try:
        GR._DEFER_ON = False
        ref = grads(False)
        GR._DEFER_ON = True
        got = grads(True)
    finally:
        GR._DEFER_ON = old
        accum.set_deferring(False)
    for n in ref:
        err = (got[n] - ref[n]).norm() / ref[n].norm().clamp_min(1e-30)
        assert err < 1e-2, (n, float(err))
