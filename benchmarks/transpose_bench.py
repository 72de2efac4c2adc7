#!/usr/bin/env python3
"""bf16 2-D transpose (transpose.hip pa_transpose2d) at the LLaMA-7B dW shapes:
achieved HBM bandwidth (read + write) vs torch's strided copy."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_amd.ops import fused  # noqa: E402


def t(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


# X^T of the mixed dW (token rows), the W^T cache refresh (weight shapes), a batched case
SHAPES = [(16384, 4096), (16384, 11008), (16384, 12288), (16384, 22016), (4096, 12288), (4096, 4096),
          (4096, 22016), (11008, 4096), (4096, 32000), (1000, 520)]
for R, C in SHAPES:
    x = torch.randn(R, C, device="cuda").to(torch.bfloat16)
    ms = t(lambda: fused.transpose2d(x))
    mt = t(lambda: x.t().contiguous())
    assert torch.equal(fused.transpose2d(x), x.t())
    gb = 2 * x.numel() * 2 / 1e9
    print(json.dumps({"mode": os.environ.get("PA_TRANSPOSE", "1"), "group": os.environ.get("PA_TR_GROUP", "auto"),
                      "R": R, "C": C, "pa_ms": round(ms, 4), "pa_TBps": round(gb / ms, 2), "torch_ms": round(mt, 4),
                      "torch_TBps": round(gb / mt, 2)}), flush=True)
