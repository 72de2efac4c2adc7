"""Debug helper: per-gradient error of a flash-attention backward variant vs fp32."""
import math
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from paddle_amd.ops import _native as N  # noqa: E402
from paddle_amd.ops import fused as F  # noqa: E402


def run(variant, B, S, H, causal):
    torch.manual_seed(0)
    D = 128
    q, k, v = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    do = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    N.call("pa_fa_bwd_set_variant", variant)
    o = F.flash_attention(q, k, v, causal=causal)
    o.backward(do)
    N.call("pa_fa_bwd_set_variant", 4)
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    F._attn_ref(qr, kr, vr, causal, 1 / math.sqrt(D)).backward(do.float())
    out = {}
    for n, a, r in (("dq", q.grad, qr.grad), ("dk", k.grad, kr.grad), ("dv", v.grad, vr.grad)):
        err = (a.float() - r).abs()
        rel = (err.norm() / r.norm()).item()
        bad = (err > 0.05 * r.abs().max()).nonzero()
        out[n] = (round(rel, 4), bad[:4].tolist() if len(bad) else [])
    print(variant, B, S, H, causal, out, flush=True)


for cfg in [(1, 128, 1, False), (1, 128, 1, True), (1, 256, 1, True), (2, 384, 2, True)]:
    for var in (1, 3, 4):
        run(var, *cfg)
