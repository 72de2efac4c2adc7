#!/usr/bin/env python3
"""dW GEMMs of the LLaMA-7B step (T = 16384 tokens): the hand-written kernel's
forms (MN x MN with tr_b16 reads; X transposed + mixed) against hipBLASLt through
torch (bf16 operands, fp32 output: torch.mm(..., out_dtype=fp32), the same
accumulate-precision contract).  Median of repetitions, TF/s per form."""
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


T = 16384
for name, (K, N) in {"qkv": (4096, 12288), "o": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096)}.items():
    x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
    xt = x.t().contiguous()
    mg = torch.zeros(K, N, device="cuda", dtype=torch.float32)
    fl = 2.0 * T * K * N
    res = {"shape": name}
    forms = {
        "pa_mn_acc": lambda: G.gemm(x, dy, K, N, T, a_kmaj=False, b_kmaj=False, out=mg, accumulate=True),
        "pa_tx_acc": lambda: G.gemm(xt, dy, K, N, T, a_kmaj=True, b_kmaj=False, out=mg, accumulate=True),
        "hipblaslt_f32out": lambda: torch.mm(x.t(), dy, out_dtype=torch.float32),
        "hipblaslt_bf16out": lambda: torch.mm(x.t(), dy),
    }
    for k, f in forms.items():
        try:
            res[k + "_tf"] = round(fl / timeit(f) / 1e9, 1)
        except Exception as e:  # an unsupported combination on this build
            res[k + "_err"] = str(e)[:80]
    # accuracy of the vendor fp32-out path vs ours
    mg.zero_()
    G.gemm(x, dy, K, N, T, a_kmaj=False, b_kmaj=False, out=mg, accumulate=False)
    try:
        ref = torch.mm(x.t(), dy, out_dtype=torch.float32)
        res["rel_diff"] = float(((mg - ref).norm() / ref.norm()).item())
    except Exception:
        pass
    print(json.dumps(res), flush=True)
    del x, dy, xt, mg
    torch.cuda.empty_cache()
