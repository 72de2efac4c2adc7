"""In-process A/B of a pa_gemm_set_* switch (0 vs 1) on the LLaMA-7B step's GEMM
forms, interleaved rounds (guide §5.4 rule 24), outputs compared bit for bit.
usage: gemm_flag_ab.py pa_gemm_set_epi_bar"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_amd.ops import _native as N  # noqa: E402
from paddle_amd.ops import gemm as G  # noqa: E402

T = 16384
SHAPES = {"qkv": (4096, 12288), "o": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096)}
setter = getattr(N.lib(), sys.argv[1])


def timeit(fn, reps=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for name, (K, Nn) in SHAPES.items():
    x = (torch.rand(T, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(K, Nn, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
    dy = (torch.rand(T, Nn, device="cuda") * 2 - 1).to(torch.bfloat16)
    wt = w.t().contiguous()
    mg = torch.zeros(K, Nn, device="cuda")
    forms = {"fwd": lambda: G.gemm(x, wt, T, Nn, K, a_kmaj=True, b_kmaj=True),
             "dx": lambda: G.gemm(dy, w, T, K, Nn, a_kmaj=True, b_kmaj=True),
             "dw_mn": lambda: G.linear_dw(x, dy, out=mg, accumulate=False)}
    for form, f in forms.items():
        outs = []
        for v in (0, 1):
            setter(v)
            outs.append(f().clone())
        same = bool(torch.equal(outs[0], outs[1]))
        res = {0: [], 1: []}
        for _ in range(5):
            for v in (0, 1):
                setter(v)
                f()
                res[v].append(timeit(f))
        med = {k: sorted(t)[len(t) // 2] for k, t in res.items()}
        flop = 2.0 * T * K * Nn
        print(json.dumps({"switch": sys.argv[1], "shape": name, "form": form, "off_ms": round(med[0], 4),
                          "on_ms": round(med[1], 4), "on_tflops": round(flop / med[1] / 1e9, 1),
                          "on_speedup": round(med[0] / med[1], 4), "identical": same}), flush=True)
    del x, w, dy, wt, mg
    torch.cuda.empty_cache()
setter(1)
