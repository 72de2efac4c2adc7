#!/usr/bin/env python3
"""Every way of laying out the weight-gradient GEMM dW[K,N] (+)= X^T dY for the
LLaMA-7B linears (T = 16384 tokens): operands as given or re-laid out token-inner
by the HIP transpose, result written row-major or through its transposed view.
Times include the transposes.  Median of interleaved repetitions."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_amd.ops import fused as F  # noqa: E402


def timeit(fn, reps=12, warm=3):
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


T = 16384
shapes = {"qkv": (4096, 12288), "o": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096),
          "lm_head": (4096, 32000)}
tr = F.transpose2d
for name, (K, N) in shapes.items():
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    g = torch.zeros(K, N, device="cuda", dtype=torch.bfloat16)
    gt = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)   # storage of the transposed result
    forms = {
        "TN(x.t,dy)": lambda: g.addmm_(x.t(), dy),
        "NN(trx,dy)": lambda: g.addmm_(tr(x), dy),
        "NT(trx,trdy.t)": lambda: g.addmm_(tr(x), tr(dy).t()),
        "T.TN(dy.t,x)": lambda: gt.addmm_(dy.t(), x),
        "T.NN(trdy,x)": lambda: gt.addmm_(tr(dy), x),
        "T.NT(trdy,trx.t)": lambda: gt.addmm_(tr(dy), tr(x).t()),
    }
    res = {k: round(timeit(f), 4) for k, f in forms.items()}
    best = min(res, key=res.get)
    print(json.dumps({"shape": name, "K": K, "N": N, **res, "best": best}), flush=True)
