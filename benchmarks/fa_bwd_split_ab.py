"""A/B of the flash-attention backward on the production path (rotary + attention
backward into the packed dqkv gradient, LLaMA-7B shape B8 H32 S2048 D128 causal):
the two-kernel split backward (fa_bwd_split.hip) vs the round-5 fused kernel with
per-key-block dQ slabs + the dQ-reduce/rotary pass + the dK rotary pass.
Interleaved rounds, outputs compared.  Prints one JSON line per arm."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_amd.ops import fused as F  # noqa: E402

B, H, S, D = [int(x) for x in os.environ.get("FA_SHAPE", "8,32,2048,128").split(",")]
Hk = int(os.environ.get("FA_HK", H))
torch.manual_seed(0)
dev = "cuda"
nh = H + 2 * Hk
packed = torch.randn(B, S, nh * D, device=dev, dtype=torch.bfloat16)
cos, sin = F.rope_tables(S, D, device=dev)
p4 = packed.view(B, S, nh, D)
scale = 1 / math.sqrt(D)
o, lse = F._fa_fwd(p4[:, :, :H], p4[:, :, H:H + Hk], p4[:, :, H + Hk:], True, scale)
do = torch.randn(B, S, H * D, device=dev, dtype=torch.bfloat16)
flop_bwd = 10 * B * H * S * S * D / 2  # 5 GEMMs, causal half


def run(split, variant=1):
    F._FA_SPLIT = split
    from paddle_amd.ops import _native as N
    N.lib().pa_fa_bwd_split_set_variant(variant)
    return F._rope_attn_backward(packed, o, lse, cos, sin, do, H, Hk, D, True, scale)


def timeit(fn, reps=10):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


res = {}
outs = {}
for rnd in range(3):
    for arm in ("split", "split_nopipe", "fused_v4"):
        t = timeit(lambda: run(arm != "fused_v4", 0 if arm == "split_nopipe" else 1))
        res.setdefault(arm, []).append(t)
        if rnd == 0:
            outs[arm] = run(arm != "fused_v4", 0 if arm == "split_nopipe" else 1).float()
F._FA_SPLIT = True
for arm, ts in res.items():
    print(json.dumps({"arm": arm, "shape": [B, H, Hk, S, D], "ms": [round(x, 4) for x in ts],
                      "TF_equiv_best": round(flop_bwd / min(ts) / 1e9, 1)}))
a, b = outs["split"].view(B, S, nh, D), outs["fused_v4"].view(B, S, nh, D)
rel = {n: float((a[:, :, sl] - b[:, :, sl]).norm() / b[:, :, sl].norm())
       for n, sl in (("dq", slice(0, H)), ("dk", slice(H, H + Hk)), ("dv", slice(H + Hk, nh)))}
print(json.dumps({"rel_diff_split_vs_fused": rel}))
c = outs["split_nopipe"].view(B, S, nh, D)
print(json.dumps({"maxabs_pipe_vs_nopipe": float((a - c).abs().max())}))
ft = timeit(lambda: F._fa_fwd(p4[:, :, :H], p4[:, :, H:H + Hk], p4[:, :, H + Hk:], True, scale))
print(json.dumps({"fwd_ms": round(ft, 4), "fwd_TF": round(4 * B * H * S * S * D / 2 / ft / 1e9, 1)}))
