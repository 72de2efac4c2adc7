"""PMC probe: the LLaMA qkv weight gradient (MN x MN, K = 16384 tokens, fp32 +=) on
the two-wave kernel and on the one-wave-per-SIMD kernel, 3 calls each."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_amd.ops import _native as N  # noqa: E402
from paddle_amd.ops import gemm as G  # noqa: E402

T, K, Nn = 16384, 4096, 12288
x = (torch.rand(T, K, device="cuda") * 2 - 1).to(torch.bfloat16)
dy = (torch.rand(T, Nn, device="cuda") * 2 - 1).to(torch.bfloat16)
mg = torch.zeros(K, Nn, device="cuda")
for v in (0, 1):
    N.lib().pa_gemm_set_dw1w(v)
    for _ in range(3):
        G.gemm(x, dy, K, Nn, T, a_kmaj=False, b_kmaj=False, out=mg, accumulate=True)
torch.cuda.synchronize()
N.lib().pa_gemm_set_dw1w(0)
