"""A/B of the persistent GEMM's start stagger (pa_gemm_set_stagger) on the LLaMA-7B
step GEMMs (T = 16384 tokens): forward (K-major x K-major via the cached W^T),
dX, and dW (both MN-major, fp32 += into main_grad), interleaved per repetition,
median of 7.  Hypothesis under test: the persistent grid's CUs run identical tile
sequences in lockstep, so all epilogues hit HBM in the same few microseconds."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_amd.ops import _native as N  # noqa: E402
from paddle_amd.ops import gemm as G  # noqa: E402

T = 16384
SHAPES = {"qkv": (4096, 12288), "o": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096)}
STAGGERS = [int(s) for s in os.environ.get("STAGGERS", "0,1,2,4,8").split(",")]
out = os.environ.get("OUT", "gpurun_out/gemm_stagger_ab.jsonl")
lib = N.lib()


def timed(fn, reps=3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


rows = []
for name, (K, Nn) in SHAPES.items():
    x = (torch.rand(T, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    wt = ((torch.rand(Nn, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
    dy = (torch.rand(T, Nn, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = wt.t().contiguous()  # the [in, out] weight: dX reads it K-major
    mg = torch.zeros(K, Nn, device="cuda")
    forms = {
        "fwd": lambda: G.gemm(x, wt, T, Nn, K, a_kmaj=True, b_kmaj=True),
        "dx": lambda: G.gemm(dy, w, T, K, Nn, a_kmaj=True, b_kmaj=True),
        "dw": lambda: G.linear_dw(x, dy, out=mg, accumulate=True),
    }
    for form, fn in forms.items():
        fn()
        res = {s: [] for s in STAGGERS}
        for _ in range(7):
            for s in STAGGERS:
                lib.pa_gemm_set_stagger(s)
                res[s].append(timed(fn))
        lib.pa_gemm_set_stagger(0)
        med = {s: statistics.median(v) for s, v in res.items()}
        r = {"shape": name, "form": form, **{f"s{s}_ms": round(m, 4) for s, m in med.items()},
             **{f"s{s}_speedup": round(med[0] / m, 4) for s, m in med.items() if s}}
        rows.append(r)
        print(json.dumps(r), flush=True)
    del x, wt, w, dy, mg
os.makedirs(os.path.dirname(out), exist_ok=True)
with open(out, "w") as f:
    for r in rows:
        f.write(json.dumps(r) + "\n")
