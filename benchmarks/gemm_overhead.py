"""Fixed per-tile cost of pa_gemm: time vs K at a fixed 16384 x 4096 output (the
K-independent part is prologue + epilogue + launch)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_amd.ops import gemm as G  # noqa: E402

M, N = 16384, 4096
for K in (64, 128, 256, 512, 1024, 4096):
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    outf = torch.empty(M, N, device="cuda", dtype=torch.float32)
    for f32 in (False, True):
        o = outf if f32 else out
        f = lambda: G.gemm(a, b, M, N, K, a_kmaj=True, b_kmaj=True, out=o)  # noqa: E731
        f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        print(json.dumps({"K": K, "out_f32": f32, "ms": round(ms, 4), "tflops": round(2 * M * N * K / ms / 1e9, 1)}))
