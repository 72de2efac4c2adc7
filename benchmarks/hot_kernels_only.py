#!/usr/bin/env python3
"""Run each hand-written hot kernel a few times at its production shape -- a short
program for rocprofv3 --pmc passes (tools/hot_pmc.sh): bf16 GEMM (LLaMA-7B qkv
forward, K-major dW into fp32), RMSNorm fwd/bwd, softmax-CE fwd/bwd (32k vocab),
NHWC conv 3x3 (ResNet-50 stage 2) fwd/bwd, fused AdamW on a 256M-element shard."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_amd.ops import conv as C  # noqa: E402
from paddle_amd.ops import fused as F  # noqa: E402
from paddle_amd.ops import gemm as G  # noqa: E402
from paddle_amd.ops import optim  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
d = "cuda"
bf = torch.bfloat16
M, K, N = 16384, 4096, 12288
x = torch.randn(M, K, device=d).to(bf)
wt = torch.randn(N, K, device=d).to(bf)
dy_t = torch.randn(N, M, device=d).to(bf)
x_t = torch.randn(K, M, device=d).to(bf)
mg = torch.zeros(K, N, device=d, dtype=torch.float32)
h = torch.randn(M, 4096, device=d).to(bf).requires_grad_(True)
nw = torch.ones(4096, device=d).to(bf).requires_grad_(True)
logits = torch.randn(8192, 32000, device=d).to(bf).requires_grad_(True)
lab = torch.randint(0, 32000, (8192,), device=d)
cx = torch.randn(64, 56, 56, 64, device=d).to(bf).requires_grad_(True)
cw = (torch.randn(64, 64, 3, 3, device=d) * 0.05).to(bf).requires_grad_(True)
n = 1 << 28
p, g, m, v = (torch.randn(n, device=d) for _ in range(4))
v.abs_()
for _ in range(reps):
    G.gemm(x, wt, M, N, K, a_kmaj=True, b_kmaj=True)                                        # qkv fwd form
    G.gemm(x_t, dy_t, K, N, M, a_kmaj=True, b_kmaj=True, out=mg, accumulate=True)          # dW form
    y = F.rms_norm(h, nw, 1e-6)
    y.backward(torch.ones_like(y))
    loss = F.softmax_cross_entropy(logits, lab)
    loss.backward()
    co = C.conv2d_nhwc(cx, cw, None, 1, 1)
    co.backward(torch.ones_like(co))
    optim.adamw_flat(p, g, m, v, lr=1e-4, weight_decay=0.1, step=2)
torch.cuda.synchronize()
print("done")
