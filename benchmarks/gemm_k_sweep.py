"""Per-tile fixed cost of the bf16 MFMA GEMM: time vs K at a fixed 16384 x 4096
output (1024 tiles of 256 x 256 = 4 per CU), both operands K-major, for bf16 out
and fp32 += out.  Fitting t(K) = a + b * K separates the per-tile fixed cost (a:
prologue, pipeline fill, epilogue) from the k-loop rate (b).  Also the same shapes
with one tile per block (non-persistent grid) for comparison."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_amd.ops import _native as N  # noqa: E402
from paddle_amd.ops import gemm as G  # noqa: E402


def timeit(fn, reps=10):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


M, Nn = 16384, 4096
out = os.environ.get("OUT", "gpurun_out/gemm_k_sweep.jsonl")
os.makedirs(os.path.dirname(out), exist_ok=True)
b = ((torch.rand(Nn, 16384, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
a = (torch.rand(M, 16384, device="cuda") * 2 - 1).to(torch.bfloat16)
c32 = torch.zeros(M, Nn, device="cuda")
rows = []
for pers in (1, 0):
    N.lib().pa_gemm_set_persistent(pers)
    for K in (1024, 2048, 4096, 8192, 16384):
        ak, bk = a[:, :K].contiguous(), b[:, :K].contiguous()
        t16 = timeit(lambda: G.gemm(ak, bk, M, Nn, K, a_kmaj=True, b_kmaj=True))
        t32 = timeit(lambda: G.gemm(ak, bk, M, Nn, K, a_kmaj=True, b_kmaj=True, out=c32, accumulate=True))
        fl = 2.0 * M * Nn * K
        r = {"persistent": pers, "K": K, "bf16_ms": round(t16, 4), "f32acc_ms": round(t32, 4),
             "bf16_tf": round(fl / t16 / 1e9, 1), "f32acc_tf": round(fl / t32 / 1e9, 1)}
        rows.append(r)
        print(json.dumps(r), flush=True)
N.lib().pa_gemm_set_persistent(1)
with open(out, "w") as f:
    for r in rows:
        f.write(json.dumps(r) + "\n")
# least-squares fit per (persistent, kind): t = a + b K; a / 4 = fixed cost per tile (us)
for pers in (1, 0):
    for kind in ("bf16_ms", "f32acc_ms"):
        xs = [r["K"] for r in rows if r["persistent"] == pers]
        ys = [r[kind] for r in rows if r["persistent"] == pers]
        n = len(xs)
        mx, my = sum(xs) / n, sum(ys) / n
        slope = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
        icpt = my - slope * mx
        print(json.dumps({"fit": kind, "persistent": pers, "fixed_us_per_tile": round(icpt * 1e3 / 4, 2),
                          "us_per_ktile_per_tile": round(slope * 64 * 1e3 / 4, 3)}), flush=True)
