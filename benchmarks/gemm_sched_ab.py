"""A/B of pa_gemm variants per form on the LLaMA-7B shapes, interleaved in one
process (guide §5.4 rule 24).  usage: gemm_sched_ab.py [sched|persistent]
  sched: load-section reads (0) vs in-cluster prefetch (1)
  persistent: one tile per block (0) vs persistent blocks (1)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_amd.ops import _native as N  # noqa: E402
from paddle_amd.ops import gemm as G  # noqa: E402

T = 16384
SHAPES = {"qkv": (4096, 12288), "o": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096)}


def timeit(fn, reps=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


what = sys.argv[1] if len(sys.argv) > 1 else "sched"
setter = N.lib().pa_gemm_set_sched if what == "sched" else N.lib().pa_gemm_set_persistent
default = -1 if what == "sched" else 1
for name, (K, Nn) in SHAPES.items():
    x = torch.randn(T, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(K, Nn, device="cuda") * 0.02).to(torch.bfloat16)
    dy = torch.randn(T, Nn, device="cuda").to(torch.bfloat16)
    mg = torch.zeros(K, Nn, device="cuda")
    forms = {"fwd": lambda: G.linear_fwd(x, w), "dx": lambda: G.linear_dx(dy, w),
             "dw": lambda: G.linear_dw(x, dy, out=mg, accumulate=True)}
    for form, f in forms.items():
        res = {0: [], 1: []}
        for r in range(6):
            for sch in (0, 1):
                setter(sch)
                f()
                res[sch].append(timeit(f))
        setter(default)
        med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
        print(json.dumps({"ab": what, "shape": name, "form": form, "off_ms": round(med[0], 4),
                          "on_ms": round(med[1], 4), "on_speedup": round(med[0] / med[1], 3)}), flush=True)
