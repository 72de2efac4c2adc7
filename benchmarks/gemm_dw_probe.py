"""PMC probe on the LLaMA qkv projection GEMMs (16384 x 12288 x 4096), 3 calls each:
forward (K-major x K-major), dW K-major x K-major on pre-transposed copies, and dW
MN-major x MN-major (tr_b16 reads, no copies)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_amd.ops import gemm as G  # noqa: E402

T, K, Nn = 16384, 4096, 12288
x = (torch.rand(T, K, device="cuda") * 2 - 1).to(torch.bfloat16)
w = ((torch.rand(K, Nn, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
wt = w.t().contiguous()
dy = (torch.rand(T, Nn, device="cuda") * 2 - 1).to(torch.bfloat16)
xt, dyt = x.t().contiguous(), dy.t().contiguous()
mg = torch.zeros(K, Nn, device="cuda")
for _ in range(3):
    G.gemm(x, wt, T, Nn, K, a_kmaj=True, b_kmaj=True)
    G.gemm(xt, dyt, K, Nn, T, a_kmaj=True, b_kmaj=True, out=mg, accumulate=True)
    G.linear_dw(x, dy, out=mg, accumulate=True)
torch.cuda.synchronize()
