"""Interleaved A/B of the flash-attention forward kernels (pa_fa_fwd_set_variant 1 vs 2)
at the LLaMA-7B attention shape (B8 H32 S2048 D128, causal), outputs compared."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_amd.ops import _native as N  # noqa: E402
from paddle_amd.ops import fused as F  # noqa: E402

B, H, S, D = 8, 32, 2048, 128
q, k, v = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16) for _ in range(3))
flop = 4 * B * H * S * S * D / 2


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


outs, res = {}, {}
for rnd in range(3):
    for var in [int(v) for v in os.environ.get("VARIANTS", "1,2").split(",")]:
        N.call("pa_fa_fwd_set_variant", var)
        t = timeit(lambda: F.flash_attention(q, k, v, causal=True))
        res.setdefault(var, []).append(t)
        if rnd == 0:
            outs[var] = F.flash_attention(q, k, v, causal=True).float()
N.call("pa_fa_fwd_set_variant", 2)
for var, ts in res.items():
    print(json.dumps({"variant": var, "ms": [round(x, 4) for x in ts], "TF_best": round(flop / min(ts) / 1e9, 1)}))
ks = sorted(outs)
print(json.dumps({f"max_abs_diff_v{ks[0]}_v{k}": float((outs[ks[0]] - outs[k]).abs().max()) for k in ks[1:]}))
