#!/usr/bin/env python3
"""GEMM probe on the LLaMA-7B step shapes (T = 16384 tokens):

* row-stride padding (ld = K vs K + 64 elements): do power-of-two strides camp on
  L2 / HBM channels?
* dW epilogue cost: fp32 accumulate vs fp32 overwrite vs bf16 out, same operands;
* forward with W as stored (MN-major B) vs the W^T copy (K-major B).

Interleaved, median of repetitions; prints one JSON line per (shape, variant)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_amd.ops import gemm as G  # noqa: E402


def timeit(fn, reps=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


def padded(rows, cols, pad):
    buf = torch.randn(rows, cols + pad, device="cuda", dtype=torch.bfloat16)
    return buf[:, :cols]


T = 16384
shapes = {"qkv": (4096, 12288), "o": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096)}
only = os.environ.get("PROBE_SHAPES")
if only:
    shapes = {k: v for k, v in shapes.items() if k in only.split(",")}
for name, (K, N) in shapes.items():
    res = {"shape": name}
    for pad in (0, 64):
        x = padded(T, K, pad)
        w = padded(K, N, pad)
        wt = padded(N, K, pad)
        dy = padded(T, N, pad)
        xt = padded(K, T, pad)
        mg = torch.zeros(K, N + pad, device="cuda", dtype=torch.float32)[:, :N]
        fl = 2.0 * T * K * N
        forms = {
            "fwd_kk": lambda: G.gemm(x, wt, T, N, K, a_kmaj=True, b_kmaj=True),
            "fwd_kn": lambda: G.gemm(x, w, T, N, K, a_kmaj=True, b_kmaj=False),
            "dx_kk": lambda: G.gemm(dy, w, T, K, N, a_kmaj=True, b_kmaj=True),
            "dw_mn_acc": lambda: G.gemm(x, dy, K, N, T, a_kmaj=False, b_kmaj=False, out=mg, accumulate=True),
            "dw_mn_fresh": lambda: G.gemm(x, dy, K, N, T, a_kmaj=False, b_kmaj=False, out=mg, accumulate=False),
            "dw_tx_acc": lambda: G.gemm(xt, dy, K, N, T, a_kmaj=True, b_kmaj=False, out=mg, accumulate=True),
            "dw_mn_bf16": lambda: G.gemm(x, dy, K, N, T, a_kmaj=False, b_kmaj=False),
        }
        if pad == 0:
            forms["torch_fwd"] = lambda: torch.mm(x, w)
        for k, f in forms.items():
            ms = timeit(f)
            res[f"{k}_p{pad}_tf"] = round(fl / ms / 1e9, 1)
        del x, w, wt, dy, xt, mg
        torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)
