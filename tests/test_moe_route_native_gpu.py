"""Native MoE routing / router backward (csrc/kernels/moe.hip: pa_moe_route,
pa_moe_frac, pa_moe_gate_bwd) against the torch formulations they replace: the
stable-argsort routing (all slots, compact capacity drop, GShard padded capacity)
must match index for index, and the fused router backward must match the fp32
autograd of softmax -> top-k -> renormalise + balance loss."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _torch_route(flat_e, T, k, E, cap):
    from paddle_amd.ops import moe_route as R

    keep = None if cap is None else R._rank_in_expert(flat_e) < cap
    _, src, pos, e_sorted = R.routing(flat_e, T, k, keep)
    counts = torch.bincount(e_sorted, minlength=E)
    return src, pos, e_sorted, counts


@pytest.mark.parametrize("T,k,E,cap", [(7, 1, 3, None), (1000, 2, 8, None), (4096, 2, 64, None),
                                       (3000, 4, 1024, None), (2048, 2, 16, 200), (513, 3, 5, 40)])
def test_route_matches_stable_argsort(T, k, E, cap):
    from paddle_amd.ops import moe_route as R

    g = torch.Generator().manual_seed(T + E)
    # skewed choices so capacity actually drops slots
    p = torch.rand(E, generator=g) ** 3 + 0.01
    flat_e = torch.multinomial(p, T * k, replacement=True, generator=g).cuda()
    ref = _torch_route(flat_e, T, k, E, cap)
    got = R.route(flat_e, T, k, E, cap)
    for a, b, nm in zip(ref, got, ("src", "pos", "e_sorted", "counts")):
        assert a.dtype == b.dtype or nm == "counts", nm
        assert torch.equal(a.long().cpu(), b.long().cpu()), nm


@pytest.mark.parametrize("T,k,E,cap", [(1024, 2, 8, 300), (999, 1, 16, 50), (64, 2, 4, 64)])
def test_capacity_routing_padded_layout(T, k, E, cap):
    from paddle_amd.ops import moe_route as R

    g = torch.Generator().manual_seed(cap)
    p = torch.rand(E, generator=g) ** 2 + 0.05
    flat_e = torch.multinomial(p, T * k, replacement=True, generator=g).cuda()
    src_n, pos_n = R.capacity_routing(flat_e, T, k, E, cap)
    # torch path of the same function (CPU tensors)
    src_t, pos_t = R.capacity_routing(flat_e.cpu(), T, k, E, cap)
    assert torch.equal(pos_n.cpu(), pos_t) and torch.equal(src_n.cpu(), src_t)


@pytest.mark.parametrize("renorm", [True, False])
@pytest.mark.parametrize("T,D,E,k", [(256, 64, 8, 2), (1000, 96, 64, 4), (33, 32, 5, 1)])
def test_gate_forward_backward_matches_fp32_autograd(T, D, E, k, renorm):
    from paddle_amd.distributed.fleet.moe import _TopKGateFn

    torch.manual_seed(T)
    x = torch.randn(T, D, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(D, E, device="cuda") * 0.2
    dval = torch.randn(T, k, device="cuda")
    daux = torch.tensor(0.37, device="cuda")

    xr = x.float().clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    probs = torch.softmax(xr @ wr, -1)
    val, idx = probs.topk(k, -1)
    valn = val / val.sum(-1, keepdim=True).clamp_min(1e-9) if renorm else val
    frac = torch.nn.functional.one_hot(idx[:, 0], E).float().mean(0)
    l_aux = (probs.mean(0) * frac).sum() * E
    (valn * dval).sum().add(l_aux * daux).backward()

    xn = x.clone().requires_grad_(True)
    wn = w.clone().requires_grad_(True)
    v2, i2, l2 = _TopKGateFn.apply(xn, wn, k, renorm)
    assert torch.equal(i2, idx)
    torch.testing.assert_close(v2, valn.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(l2, l_aux.detach(), rtol=1e-5, atol=1e-6)
    torch.autograd.backward([v2, l2], [dval, daux])
    torch.testing.assert_close(wn.grad, wr.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(xn.grad.float(), xr.grad, rtol=2e-2, atol=2e-3)


def test_ernie_moe_step_has_no_aten_routing_kernels():
    """The ERNIE-MoE training step's routing and router backward run on the native
    kernels: no sort / index_put_ / scatter / index_add_ left in the MoE regions."""
    import os

    os.environ["FLAGS_count_aten"] = "1"
    try:
        from paddle_amd.autograd import tape
        from paddle_amd.models.ernie_moe import ERNIE_MOE_CONFIGS, ErnieMoEConfig, ErnieMoEForCausalLM
        from paddle_amd.utils import strict

        torch.manual_seed(0)
        cfg = ErnieMoEConfig(**dict(ERNIE_MOE_CONFIGS["ernie-moe-tiny"], hidden_size=256, moe_intermediate_size=128,
                                    intermediate_size=512, grouped_experts=True, max_position_embeddings=1024))
        m = ErnieMoEForCausalLM(cfg, torch.device("cuda", 0))
        ids = torch.randint(0, cfg.vocab_size, (2, 257), device="cuda")
        with tape.recording() as t:
            loss = m(ids[:, :-1], ids[:, 1:])
        strict.reset()
        with strict.region("ernie:step"):
            with tape.recording() as t:
                loss = m(ids[:, :-1], ids[:, 1:])
            t.backward(loss)
        torch.cuda.synchronize()
        rep = strict.report()["aten_kernels"]
        bad = {k_: v for k_, v in rep.items() if any(s in k_ for s in ("sort", "index_put", "scatter", "index_add",
                                                                       "one_hot"))}
        assert not bad, rep
        assert not {k_ for k_ in rep if k_.startswith("moe:")}, rep
    finally:
        os.environ.pop("FLAGS_count_aten", None)
