"""bf16 vs fp8 (block-scaled MFMA) GEMM throughput, plain and grouped (MoE expert
shapes).  Prints one JSON line per case."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_amd.ops import fp8, gemm as G  # noqa: E402


def timeit(fn, iters=20):
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


dev = "cuda"
for M, N, K in [(8192, 8192, 8192), (16384, 4096, 4096), (8192, 11008, 4096)]:
    a = torch.randn(M, K, device=dev).to(torch.bfloat16)
    b = torch.randn(N, K, device=dev).to(torch.bfloat16)
    aq, sa = fp8.quant_rows(a)
    bq, sb = fp8.quant_rows(b)
    o = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    t16 = timeit(lambda: G.gemm(a, b, M, N, K, a_kmaj=True, b_kmaj=True, out=o))
    t8 = timeit(lambda: fp8.gemm_f8(aq, sa, bq, sb, M, N, K, out=o))
    tq = timeit(lambda: fp8.quant_rows(a))
    f = 2 * M * N * K
    print(json.dumps({"case": "plain", "M": M, "N": N, "K": K, "bf16_tf": round(f / t16 / 1e9, 1),
                      "fp8_tf": round(f / t8 / 1e9, 1), "quant_a_us": round(tq * 1e3, 1)}), flush=True)

# grouped: 64 experts x 768 tokens, ERNIE-MoE a3b shapes
E, T, H, I2 = 64, 768, 2560, 3072
counts = [T] * E
R = E * T
offs = G.group_table(torch.tensor([i * T for i in range(E + 1)], dtype=torch.int32, device=dev), E * T)
x = torch.randn(R, H, device=dev).to(torch.bfloat16)
w = (torch.randn(E, H, I2, device=dev) * 0.02).to(torch.bfloat16)
out = torch.empty(R, I2, device=dev, dtype=torch.bfloat16)
wq, ws = fp8.quant_cols_t(w)
xq, xs = fp8.quant_rows(x)
t16 = timeit(lambda: G.grouped_rows(x, w, offs, b_kmaj=False, out=out))
t8 = timeit(lambda: fp8.gemm_f8(xq, xs, wq, ws, R, I2, H, out=out, batch=E, sB=I2 * H, grp=offs, grp_mode=1))
tw = timeit(lambda: fp8.quant_cols_t(w), 5)
f = 2 * R * H * I2
print(json.dumps({"case": "grouped_gate_up", "E": E, "tokens_per_expert": T, "H": H, "N": I2,
                  "bf16_tf": round(f / t16 / 1e9, 1), "fp8_tf": round(f / t8 / 1e9, 1),
                  "weight_quant_ms": round(tw, 3)}), flush=True)
