#!/usr/bin/env python3
"""A/B of the one-wave-per-SIMD weight-gradient GEMM (gemm.hip gemm1w_kernel) against
the two-wave kernel on the LLaMA-7B dW shapes (T = 16384 tokens, fp32 main_grad +=):
  MN x MN: dW[K,N] += x[T,K]^T dY[T,N]        (both operands token-outer, as stored)
  mixed  : dW[K,N] += (x^T)[K,T] dY[T,N]      (x^T a token-contiguous copy)
Prints ms, PFLOP/s and the max |diff| between the two kernels' results, one JSON
line per (shape, form).  Interleaved medians."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_amd.ops import _native as N  # noqa: E402
from paddle_amd.ops import gemm as G  # noqa: E402


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


T = int(os.environ.get("DW_T", 16384))
shapes = {"qkv": (4096, 12288), "o": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096)}
lib = N.lib()
torch.manual_seed(0)
for name, (K, Nn) in shapes.items():
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    xt = x.t().contiguous()
    dy = torch.randn(T, Nn, device="cuda", dtype=torch.bfloat16)
    for form in ("mnmn", "mixed"):
        if form == "mnmn":
            run = lambda out: G.gemm(x, dy, K, Nn, T, a_kmaj=False, b_kmaj=False, out=out, accumulate=True)  # noqa: E731
        else:
            run = lambda out: G.gemm(xt, dy, K, Nn, T, a_kmaj=True, b_kmaj=False, out=out, accumulate=True)  # noqa: E731
        outs, ts = {}, {0: [], 1: []}
        for v in (0, 1):
            lib.pa_gemm_set_dw1w(v)
            outs[v] = torch.zeros(K, Nn, device="cuda", dtype=torch.float32)
            run(outs[v])
        torch.cuda.synchronize()
        diff = (outs[0] - outs[1]).abs().max().item()
        scale = outs[0].abs().max().item()
        for _ in range(2):
            for v in (0, 1):
                lib.pa_gemm_set_dw1w(v)
                run(outs[v])
        for _ in range(8):
            for v in (0, 1):
                lib.pa_gemm_set_dw1w(v)
                ts[v].append(timed(lambda: run(outs[v])))
        fl = 2.0 * T * K * Nn
        r = {"shape": name, "form": form, "K": K, "N": Nn, "T": T}
        for v, tag in ((0, "w2"), (1, "w1")):
            ms = statistics.median(ts[v])
            r[f"{tag}_ms"] = round(ms, 4)
            r[f"{tag}_pf"] = round(fl / ms / 1e12, 3)
        r["speedup"] = round(r["w2_ms"] / r["w1_ms"], 3)
        r["maxdiff"] = diff
        r["maxabs"] = scale
        print(json.dumps(r), flush=True)
lib.pa_gemm_set_dw1w(0)
