"""Model families on CPU: GPT (single / TP / PP with tied embeddings / TP x PP
hybrid = BASELINE's "GPT-3 TP=2 PP=2" layout at tiny scale), ERNIE-MoE (single /
expert parallel), fp8 expert GEMM numerics."""
import pytest
import torch

from dist_util import run_dist
from paddle_amd.models.ernie_moe import ERNIE_MOE_CONFIGS, ErnieMoEConfig, ErnieMoEForCausalLM
from paddle_amd.models.gpt import (GPT_CONFIGS, GPTConfig, GPTForCausalLM, GPTPretrainingCriterion,
                                   gpt_pipeline_descs, shard_gpt_state_dict)


def _gcfg(**kw):
    c = dict(GPT_CONFIGS["gpt-tiny"])
    c.update(kw)
    return GPTConfig(**c, dtype="float32")


def _batch(B=4, S=17, V=512, seed=3):
    return torch.randint(0, V, (B, S), generator=torch.Generator().manual_seed(seed))


def test_gpt_tiny_trains():
    torch.manual_seed(0)
    m = GPTForCausalLM(_gcfg(), "cpu")
    opt = torch.optim.AdamW(m.parameters(), lr=3e-3)
    b = _batch()
    losses = []
    for _ in range(15):
        loss = m(b[:, :-1], b[:, 1:])
        loss.backward()
        opt.step()
        opt.zero_grad()
        losses.append(loss.item())
    assert losses[-1] < losses[0] - 1.0


def _gpt_tp_worker(rank, world):
    from paddle_amd.distributed.fleet import TPGroup

    cfg = _gcfg()
    torch.manual_seed(0)
    full = GPTForCausalLM(cfg, "cpu")
    b = _batch()
    ref = full(b[:, :-1], b[:, 1:])
    ref.backward()
    gref = shard_gpt_state_dict({n: p.grad for n, p in full.named_parameters()}, cfg, rank, world)
    m = GPTForCausalLM(cfg, "cpu", tp=TPGroup(None))
    m.load_state_dict(shard_gpt_state_dict({k: v.detach() for k, v in full.state_dict().items()}, cfg, rank, world))
    loss = m(b[:, :-1], b[:, 1:])
    loss.backward()
    return loss.item(), ref.item(), max((p.grad - gref[n]).abs().max().item() for n, p in m.named_parameters())


def test_gpt_tensor_parallel_matches_single():
    for loss, ref, gerr in run_dist(_gpt_tp_worker, 2):
        assert abs(loss - ref) < 1e-5 and gerr < 1e-5


def _gpt_pp_ref(M, steps):
    from paddle_amd.distributed.fleet.pipeline import PipelineLayer

    cfg = _gcfg(num_hidden_layers=4)
    crit = GPTPretrainingCriterion()
    model = PipelineLayer(gpt_pipeline_descs(cfg, "cpu"), num_stages=1, loss_fn=crit, seed=5)
    opt = torch.optim.SGD(model.parameters(), lr=0.5)
    losses = []
    for s in range(steps):
        b = _batch(B=8, seed=s)
        tot = 0.0
        for mb in b.chunk(M):
            loss = crit(model(mb[:, :-1]), mb[:, 1:]) / M
            loss.backward()
            tot += loss.item()
        opt.step()
        opt.zero_grad()
        losses.append(tot)
    return losses, {n: p.detach().clone() for n, p in model.named_parameters()}


def _gpt_hybrid_worker(rank, world, mp, pp, M, steps):
    from paddle_amd.distributed.fleet import DistributedStrategy, TPGroup, fleet
    from paddle_amd.distributed.fleet.pipeline import PipelineLayer

    st = DistributedStrategy()
    st.hybrid_configs = {"dp_degree": 1, "mp_degree": mp, "pp_degree": pp}
    st.pipeline_configs = {"accumulate_steps": M}
    fleet.init(is_collective=True, strategy=st)
    hcg = fleet.get_hybrid_communicate_group()
    cfg = _gcfg(num_hidden_layers=4)
    tp = TPGroup(hcg.get_model_parallel_group())
    layer = PipelineLayer(gpt_pipeline_descs(cfg, "cpu", tp), hcg=hcg, loss_fn=GPTPretrainingCriterion(tp), seed=5)
    if mp > 1:
        # same weights as the single-process reference: build the full stage, shard it
        full = PipelineLayer(gpt_pipeline_descs(cfg, "cpu"), hcg=hcg, loss_fn=None, seed=5)
        sd = shard_gpt_state_dict({k: v.detach() for k, v in full.state_dict().items()}, cfg,
                                  hcg.get_model_parallel_rank(), mp)
        layer.load_state_dict(sd)
    model = fleet.distributed_model(layer)
    opt = torch.optim.SGD(model.parameters(), lr=0.5)
    losses = [model.train_batch((_batch(B=8, seed=s)[:, :-1], _batch(B=8, seed=s)[:, 1:]), opt).item()
              for s in range(steps)]
    lo = layer.bounds[hcg.get_stage_id()]
    params = {}
    for n, p in layer.named_parameters():
        parts = n.split(".")
        params[".".join(["run_function", str(lo + int(parts[1]))] + parts[2:])] = p.detach().clone()
    return losses, params, hcg.get_model_parallel_rank()


@pytest.mark.parametrize("mp,pp", [(1, 2), (2, 2)])
def test_gpt_hybrid_tp_pp_matches_single(mp, pp):
    M, steps = 4, 2
    ref_losses, ref = _gpt_pp_ref(M, steps)
    cfg = _gcfg(num_hidden_layers=4)
    for losses, params, mp_rank in run_dist(_gpt_hybrid_worker, mp * pp, mp, pp, M, steps):
        for a, b in zip(losses, ref_losses):
            assert abs(a - b) < 1e-4, (losses, ref_losses)
        want = shard_gpt_state_dict(ref, cfg, mp_rank, mp)
        last = len(gpt_pipeline_descs(cfg)) - 1
        for n, p in params.items():
            # the tied head layer is the embedding's second occurrence (index `last` -> 0)
            if n.startswith(f"run_function.{last}.layer.") and not n.endswith("word_embeddings"):
                continue  # only the tied weight is shared; the head copy's other params are unused
            key = n.replace(f"run_function.{last}.layer.", "run_function.0.layer.")
            assert torch.allclose(p, want[key], atol=1e-5), n


def _ecfg(**kw):
    c = dict(ERNIE_MOE_CONFIGS["ernie-moe-tiny"])
    c.update(kw)
    return ErnieMoEConfig(**c, dtype="float32")


def test_ernie_moe_tiny_trains():
    torch.manual_seed(0)
    m = ErnieMoEForCausalLM(_ecfg(), "cpu")
    opt = torch.optim.AdamW(m.parameters(), lr=3e-3)
    b = _batch()
    losses = []
    for _ in range(12):
        loss = m(b[:, :-1], b[:, 1:])
        loss.backward()
        opt.step()
        opt.zero_grad()
        losses.append(loss.item())
    assert losses[-1] < losses[0] - 1.0
    assert any(l.is_moe for l in m.layers) and not m.layers[0].is_moe


def _ernie_ep_worker(rank, world):
    cfg = _ecfg()
    torch.manual_seed(0)
    ref = ErnieMoEForCausalLM(cfg, "cpu")
    torch.manual_seed(0)
    m = ErnieMoEForCausalLM(cfg, "cpu", ep_group=torch.distributed.group.WORLD)
    b = _batch(seed=11 + rank)
    l_ref = ref(b[:, :-1], b[:, 1:])
    l_ep = m(b[:, :-1], b[:, 1:])
    l_ep.backward()
    return l_ref.item(), l_ep.item(), m.layers[1].moe.n_local


def test_ernie_moe_expert_parallel_matches_single():
    for l_ref, l_ep, n_local in run_dist(_ernie_ep_worker, 2):
        assert n_local == 2
        assert abs(l_ref - l_ep) < 1e-5


def test_fp8_linear_numerics_and_grads():
    from paddle_amd.ops.fp8 import fp8_linear

    torch.manual_seed(0)
    x = torch.randn(64, 128, requires_grad=True)
    w = torch.nn.Parameter(torch.randn(128, 96) * 0.05)
    y = fp8_linear(x, w)
    ref = x @ w
    rel = ((y - ref).norm() / ref.norm()).item()
    assert rel < 0.06  # e4m3 has a 3-bit mantissa
    y.sum().backward()
    dx_ref = torch.ones(64, 96) @ w.t()
    assert ((x.grad - dx_ref).norm() / dx_ref.norm()).item() < 0.06  # fp8 dgrad (per-row scaled)
    assert torch.allclose(w.grad, x.detach().t() @ torch.ones(64, 96), atol=1e-4)  # wgrad unquantised
    with torch.no_grad():
        w.mul_(2.0)  # version bump -> re-quantised weight
    assert ((fp8_linear(x, w) - 2 * y).abs().max() / y.abs().max()).item() < 0.1


def test_ernie_moe_grouped_experts_match_per_expert_loop():
    """The grouped (padded batched-GEMM) expert path equals the per-expert loop:
    same init per expert, same loss and gradients."""
    ids = _batch(seed=3)
    out = []
    for grouped in (False, True):
        torch.manual_seed(0)
        m = ErnieMoEForCausalLM(_ecfg(grouped_experts=grouped), "cpu")
        loss = m(ids[:, :-1], ids[:, 1:])
        loss.backward()
        ex = m.layers[1].moe.experts
        assert m.layers[1].moe.grouped == grouped
        gu = ex.gate_up.grad[1] if grouped else ex[1].gate_up.grad
        dn = ex.down.grad[3] if grouped else ex[3].down.grad
        out.append((loss.detach(), gu, dn, m.embed_tokens.grad))
    for a, b in zip(*out):
        assert torch.allclose(a, b, atol=1e-6, rtol=1e-5)
