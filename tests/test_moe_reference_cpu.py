"""``MoELayer`` against the per-token dense formula:

    out_t = sum_k gate_k(t) * expert_{idx_k(t)}(x_t)

with fp32 experts evaluated token by token -- no routing, sorting, dispatch or
combine code shared with the layer.  Covers the per-expert loop, the grouped
(stacked-weight) experts, the sync-free fixed-capacity layout (with and without
dropped slots) and expert parallelism over 2 gloo ranks.  A layer that mixed
token positions (e.g. a dispatch / combine permutation bug) fails here."""
import pytest
import torch
import torch.nn.functional as F

from dist_util import run_dist
from paddle_amd.distributed.fleet.moe import MoELayer, TopKGate
from paddle_amd.models.ernie_moe import GroupedSwiGLUExperts, SwiGLUExpert

H, I, E, K = 16, 8, 4, 2


def _seed(e):
    return 1000 + e


def _loop_experts(experts):
    out = []
    for e in experts:
        torch.manual_seed(_seed(e))
        out.append(SwiGLUExpert(H, I, "cpu", torch.float32, 0.2))
    return out


def _dense_ref(x, val, idx, weights, keep=None):
    """weights[e] = (gate_up [H, 2I], down [I, H]); keep [T, K] bool (capacity drops)."""
    T = x.shape[0]
    out = torch.zeros(T, H, dtype=torch.float64)
    for t in range(T):
        for j in range(val.shape[1]):
            if keep is not None and not keep[t, j]:
                continue
            gu, dn = weights[int(idx[t, j])]
            h = x[t].double() @ gu.double()
            a = F.silu(h[:I]) * h[I:]
            out[t] += float(val[t, j]) * (a @ dn.double())
    return out


def _weights_of(experts):
    return {e: (m.gate_up.detach(), m.down.detach()) for e, m in zip(range(len(experts)), experts)}


def _capacity_keep(idx, cap):
    """Slot (t, j) is kept when it is among the first ``cap`` slots of its expert in
    flat slot order t * K + j (GShard drop rule)."""
    flat = idx.reshape(-1)
    seen, keep = {}, torch.zeros(flat.numel(), dtype=torch.bool)
    for s in range(flat.numel()):
        e = int(flat[s])
        seen[e] = seen.get(e, 0) + 1
        keep[s] = seen[e] <= cap
    return keep.view(idx.shape)


def _gate():
    torch.manual_seed(7)
    g = TopKGate(H, E, K, "gshard")
    with torch.no_grad():
        g.weight.normal_(0, 0.5)
    return g


@pytest.mark.parametrize("layout", ["loop", "grouped"])
@pytest.mark.parametrize("capacity", [None, 100.0, 0.5])
def test_moe_layer_matches_per_token_dense_formula(layout, capacity):
    torch.manual_seed(0)
    T = 24
    x = torch.randn(T, H)
    if layout == "loop":
        experts = _loop_experts(range(E))
        weights = _weights_of(experts)
    else:
        experts = GroupedSwiGLUExperts(H, I, range(E), "cpu", torch.float32, 0.2, _seed)
        weights = {e: (experts.gate_up[e].detach(), experts.down[e].detach()) for e in range(E)}
    moe = MoELayer(H, experts, gate=_gate(), capacity_factor=capacity)
    with torch.no_grad():
        y = moe(x)
        val, idx, _ = moe.gate(x)
    keep = None
    if capacity is not None:
        keep = _capacity_keep(idx, max(1, int(capacity * T * K / E)))
        if capacity < 1:
            assert not bool(keep.all())  # the case really drops slots
    ref = _dense_ref(x, val, idx, weights, keep)
    assert torch.allclose(y.double(), ref, atol=1e-5, rtol=1e-5), (y.double() - ref).abs().max()
    # position independence: permuting the tokens permutes the output
    perm = torch.randperm(T)
    with torch.no_grad():
        yp = moe(x[perm])
    if capacity is None or capacity >= 100:
        assert torch.allclose(yp, y[perm], atol=1e-6)


def _ep_worker(rank, world, capacity):
    from paddle_amd.parallel import comm

    comm.init_parallel_env()
    nl = E // world
    experts = GroupedSwiGLUExperts(H, I, range(rank * nl, (rank + 1) * nl), "cpu", torch.float32, 0.2, _seed)
    moe = MoELayer(H, experts, gate=_gate(), group=None, capacity_factor=capacity)
    torch.manual_seed(100 + rank)
    x = torch.randn(20, H)
    with torch.no_grad():
        y = moe(x)
        val, idx, _ = moe.gate(x)
    return x, y, val, idx


@pytest.mark.parametrize("capacity", [None, 100.0])
def test_moe_layer_expert_parallel_matches_dense_formula(capacity):
    full = GroupedSwiGLUExperts(H, I, range(E), "cpu", torch.float32, 0.2, _seed)
    weights = {e: (full.gate_up[e].detach(), full.down[e].detach()) for e in range(E)}
    for x, y, val, idx in run_dist(_ep_worker, 2, capacity):
        ref = _dense_ref(x, val, idx, weights)
        assert torch.allclose(y.double(), ref, atol=1e-5, rtol=1e-5), (y.double() - ref).abs().max()
