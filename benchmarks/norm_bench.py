#!/usr/bin/env python3
"""RMSNorm (+ fused residual) forward / backward at the LLaMA-7B step shape
([16384, 4096] bf16): ms and effective HBM bandwidth."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_amd.ops import fused as F  # noqa: E402


def timeit(fn, n=20, w=3):
    for _ in range(w):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


T, H = 16384, 4096
x = torch.randn(T, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
r = torch.randn(T, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
w = torch.ones(H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
dy = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
dh = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
fwd = timeit(lambda: F.rms_norm(x, w, 1e-6, residual=r))
y, h = F.rms_norm(x, w, 1e-6, residual=r)
tot = timeit(lambda: torch.autograd.grad((y, h), (x, r, w), (dy, dh), retain_graph=True))
nb = T * H * 2
print(json.dumps({"fwd_ms": round(fwd, 4), "fwd_TBps": round(4 * nb / fwd / 1e9, 2),
                  "bwd_ms": round(tot, 4), "bwd_TBps_min_traffic": round(4 * nb / tot / 1e9, 2)}))
