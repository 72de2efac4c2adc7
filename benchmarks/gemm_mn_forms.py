"""Transposed-read (MN-major) GEMM forms vs the K-major forms the LLaMA step runs
today, on the LLaMA-7B shapes (T = 16384 tokens), interleaved in one process:
  dw_kk : dW = (X^T)(dY^T)^T on two HIP-transposed copies, both K-major (times
          INCLUDE the two transposes: this is the production path)
  dw_mn : dW = X^T dY straight from the stored layouts, both MN-major (tr_b16 reads)
  dw_tx / dw_tdy: one operand transposed (x or dY) + the mixed form (times include it)
  fwd_kk: y = x W via the cached K-major W^T        fwd_kn: B = W MN-major
each MN form under both schedules (pa_gemm_set_sched 0 / 1)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_amd.ops import _native as N  # noqa: E402
from paddle_amd.ops import gemm as G  # noqa: E402
from paddle_amd.ops.fused import transpose2d  # noqa: E402

T = 16384
SHAPES = {"qkv": (4096, 12288), "o": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096)}
setsched = N.lib().pa_gemm_set_sched


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
    forms = {
        "dw_kk": (-1, lambda: G.gemm(transpose2d(x), transpose2d(dy), K, Nn, T, a_kmaj=True, b_kmaj=True, out=mg,
                                     accumulate=True)),
        "dw_tx": (-1, lambda: G.gemm(transpose2d(x), dy, K, Nn, T, a_kmaj=True, b_kmaj=False, out=mg,
                                     accumulate=True)),
        "dw_tdy": (-1, lambda: G.gemm(x, transpose2d(dy), K, Nn, T, a_kmaj=False, b_kmaj=True, out=mg,
                                      accumulate=True)),
        "dw_mn_s0": (0, lambda: G.linear_dw(x, dy, out=mg, accumulate=True)),
        "dw_mn_s1": (1, lambda: G.linear_dw(x, dy, out=mg, accumulate=True)),
        "fwd_kk": (-1, lambda: G.gemm(x, wt, T, Nn, K, a_kmaj=True, b_kmaj=True)),
        "fwd_kn_s0": (0, lambda: G.linear_fwd(x, w)),
        "fwd_kn_s1": (1, lambda: G.linear_fwd(x, w)),
    }
    res = {k: [] for k in forms}
    for _ in range(5):
        for k, (sch, f) in forms.items():
            setsched(sch)
            f()
            res[k].append(timeit(f))
    setsched(-1)
    flop = 2.0 * T * K * Nn
    med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    print(json.dumps({"shape": name, **{k + "_ms": round(v, 4) for k, v in med.items()},
                      **{k + "_tf": round(flop / v / 1e9, 1) for k, v in med.items()}}), flush=True)
    del x, w, dy, wt, mg
    torch.cuda.empty_cache()
