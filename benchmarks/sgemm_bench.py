#!/usr/bin/env python3
"""Exact-fp32 MFMA GEMM (convnd.hip pa_sgemm) vs torch.mm (hipBLASLt) fp32 on
Fluid-sized shapes; one JSON line per shape (TFLOP/s, max rel error vs fp64)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_amd.ops import convnd as C  # noqa: E402


def bench(fn, iters=20):
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


for M, N, K in [(4096, 4096, 4096), (8192, 8192, 2048), (1024, 4096, 1024), (128, 2048, 512), (6272, 64, 576)]:
    a = torch.randn(M, K, device="cuda")
    b = torch.randn(K, N, device="cuda")
    c = torch.empty(M, N, device="cuda")
    t_n = bench(lambda: C.sgemm(a, K, 1, b, N, 1, c, N, M, N, K))
    t_t = bench(lambda: torch.mm(a, b, out=c))
    C.sgemm(a, K, 1, b, N, 1, c, N, M, N, K)
    ref = a.double() @ b.double()
    err = ((c.double() - ref).abs().max() / ref.abs().max()).item()
    fl = 2 * M * N * K
    print(json.dumps({"M": M, "N": N, "K": K, "pa_sgemm_tflops": round(fl / t_n / 1e9, 1),
                      "torch_mm_tflops": round(fl / t_t / 1e9, 1), "pa_ms": round(t_n, 4), "torch_ms": round(t_t, 4),
                      "max_rel_err": err}), flush=True)
