#!/usr/bin/env python3
"""Run only the flash-attention forward kernel a few times -- a short program for
rocprofv3 --pmc passes (LLaMA-7B shape B8 H32 S2048 D128, causal)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_amd.ops import fused as F  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
B, H, S, D = 8, 32, 2048, 128
q, k, v = (torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16) for _ in range(3))
for _ in range(reps):
    F.flash_attention(q, k, v, causal=True)
torch.cuda.synchronize()
print("done")
