#!/usr/bin/env python3
"""Run only the flash-attention backward kernel (variant from argv) a few times --
a short program for rocprofv3 --pmc passes (LLaMA-7B shape B8 H32 S2048 D128)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_amd.ops import _native as N  # noqa: E402
from paddle_amd.ops import fused as F  # noqa: E402

variant = int(sys.argv[1]) if len(sys.argv) > 1 else 3
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
B, H, S, D = 8, 32, 2048, 128
q, k, v = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
do = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
N.call("pa_fa_bwd_set_variant", variant)
o = F.flash_attention(q, k, v, causal=True)
for _ in range(reps):
    torch.autograd.grad(o, (q, k, v), do, retain_graph=True)
torch.cuda.synchronize()
print("done", variant)
