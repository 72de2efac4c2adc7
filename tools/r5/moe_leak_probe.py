"""Localise the ERNIE-MoE position leak: per stage, (a) determinism (same input
twice) and (b) dependence of positions < cut on tokens >= cut."""
import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
from paddle_amd.models.ernie_moe import ERNIE_MOE_CONFIGS, ErnieMoEConfig, ErnieMoEForCausalLM, ErnieMoEDecoderLayer
from paddle_amd.ops import moe_route as R
from paddle_amd import ops

torch.manual_seed(0)
cfg = ErnieMoEConfig(**dict(ERNIE_MOE_CONFIGS["ernie-moe-a3b-8l"], num_hidden_layers=2, grouped_experts=True))
layer = ErnieMoEDecoderLayer(cfg, "cuda", layer_idx=1)
moe = layer.moe
S, H, cut = 2048, cfg.hidden_size, 1111
x = (torch.randn(S, H, device="cuda") ).to(torch.bfloat16)
x2 = x.clone(); x2[cut:] = torch.randn(S - cut, H, device="cuda").to(torch.bfloat16)

def d(a, b, n=cut):
    return (a[:n].float() - b[:n].float()).abs().max().item()

with torch.no_grad():
    # gate stage
    l1 = x.float() @ moe.gate.weight.float(); l1b = x.float() @ moe.gate.weight.float(); l2 = x2.float() @ moe.gate.weight.float()
    print("gate logits: rerun", d(l1, l1b, S), "perturbed", d(l1, l2))
    from paddle_amd.utils import strict
    with strict.region("probe"):
        m1 = x.float() @ moe.gate.weight.float(); m1b = x.float() @ moe.gate.weight.float(); m2 = x2.float() @ moe.gate.weight.float()
    print("gate logits (native region): rerun", d(m1, m1b, S), "perturbed", d(m1, m2), "vs torch", d(m1, l1, S))
    v1, i1, _ = moe.gate(x); v1b, i1b, _ = moe.gate(x); v2, i2, _ = moe.gate(x2)
    print("gate vals: rerun", d(v1, v1b, S), "perturbed", d(v1, v2), "idx equal<cut", torch.equal(i1[:cut], i2[:cut]),
          "idx rerun equal", torch.equal(i1, i1b))
    # torch reference gate (no native region)
    p = torch.softmax(l1, -1); rv, ri = p.topk(cfg.top_k, -1); rv = rv / rv.sum(-1, keepdim=True)
    print("gate vs torch topk: idx equal", torch.equal(ri, i1), "val diff", (rv - v1).abs().max().item())
    # full moe
    y1 = moe(x); y1b = moe(x); y2 = moe(x2)
    print("moe out: rerun", d(y1, y1b, S), "perturbed", d(y1, y2))
    # per-token dense reference with the SAME routing
    k = cfg.top_k
    gu, dn = moe.experts.gate_up.float(), moe.experts.down.float()
    ref = torch.zeros(S, H, device="cuda")
    for j in range(k):
        e = i1[:, j]
        h = torch.bmm(x.float().unsqueeze(1), gu[e]).squeeze(1)
        I = h.shape[1] // 2
        a = torch.nn.functional.silu(h[:, :I]) * h[:, I:]
        ref += v1[:, j:j + 1].float() * torch.bmm(a.unsqueeze(1), dn[e]).squeeze(1)
    err = (y1.float() - ref).norm() / ref.norm()
    rowerr = ((y1.float() - ref).norm(dim=1) / ref.norm(dim=1))
    print("moe vs per-token dense ref: rel", err.item(), "worst row", rowerr.max().item(), "rows>5%", int((rowerr > 0.05).sum()))
    # dispatch / combine alone
    flat_e = i1.reshape(-1)
    _, src, pos, e_sorted = R.routing(flat_e, S, k)
    send = R.dispatch(x, src, pos, k)
    print("dispatch exact", torch.equal(send, x[src.long()]))
    ys = torch.randn(send.shape, device="cuda").to(torch.bfloat16)
    yc = R.combine(ys, v1.reshape(-1), pos, k)
    yr = torch.zeros(S, H, device="cuda")
    for j in range(k):
        yr += v1[:, j:j + 1].float() * ys[pos.view(S, k)[:, j].long()].float()
    print("combine vs ref", ((yc.float() - yr).norm() / yr.norm()).item())
    # grouped expert mlp alone vs per-expert fp32
    counts = torch.zeros(cfg.num_experts, dtype=torch.int64, device="cuda").index_add_(0, e_sorted, torch.ones_like(e_sorted))
    yg = moe.experts.forward_grouped(send, counts)
    offs = [0] + torch.cumsum(counts, 0).tolist()
    worst = 0.0
    for e in range(cfg.num_experts):
        a0, a1 = offs[e], offs[e + 1]
        if a1 == a0: continue
        h = send[a0:a1].float() @ gu[e]; I = h.shape[1] // 2
        r = (torch.nn.functional.silu(h[:, :I]) * h[:, I:]) @ dn[e]
        worst = max(worst, ((yg[a0:a1].float() - r).norm() / r.norm()).item())
    print("grouped experts worst per-expert rel err", worst)
    # attention part of the layer
    cos, sin = ops.rope_tables(cfg.max_position_embeddings, cfg.head_dim, cfg.rope_theta, device="cuda")
    xx = x.unsqueeze(0); xx2 = x2.unsqueeze(0)
    o1 = layer(xx, None, cos, sin); o2 = layer(xx2, None, cos, sin); o1b = layer(xx, None, cos, sin)
    print("decoder layer m: rerun", d(o1[0][0], o1b[0][0], S), "perturbed", d(o1[0][0], o2[0][0]))
    print("decoder layer h2: rerun", d(o1[1][0], o1b[1][0], S), "perturbed", d(o1[1][0], o2[1][0]))
