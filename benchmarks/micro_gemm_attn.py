#!/usr/bin/env python3
"""Micro-benchmarks used to steer kernel work (run on the MI355X box).

* LLaMA-7B linear layers at 16384 tokens: forward (NN), dX (NT), dX via an explicit
  transposed weight copy (T + NN), dW (TN) -- hipBLASLt, bf16.
* Flash attention fwd / bwd (paddle_amd gfx950 kernels) vs torch SDPA on the same
  random data, B=8 H=32 S=2048 D=128 causal.
Interleaved repetitions in one process (guide §5.4 rule 24); median reported.
"""
import json
import statistics
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps=20, warm=3):
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


def gemms():
    dev = "cuda"
    N = 16384
    res = {}
    for name, (K, M) in {"qkv": (4096, 12288), "o": (4096, 4096), "gate_up": (4096, 22016),
                         "down": (11008, 4096), "lm_head": (4096, 32000)}.items():
        x = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(K, M, device=dev, dtype=torch.bfloat16) * 0.02
        dy = torch.randn(N, M, device=dev, dtype=torch.bfloat16)
        g = torch.zeros(K, M, device=dev, dtype=torch.bfloat16)
        flop = 2 * N * K * M
        t_fwd = timeit(lambda: torch.matmul(x, w))
        t_dx = timeit(lambda: torch.matmul(dy, w.t()))
        t_dxT = timeit(lambda: torch.matmul(dy, w.t().contiguous()))
        t_tr = timeit(lambda: w.t().contiguous())
        t_dw = timeit(lambda: g.addmm_(x.t(), dy))
        res[name] = {k: round(v, 3) for k, v in dict(fwd_ms=t_fwd, dx_nt_ms=t_dx, dx_transpose_nn_ms=t_dxT,
                                                     transpose_ms=t_tr, dw_tn_acc_ms=t_dw).items()}
        res[name]["fwd_TF"] = round(flop / t_fwd / 1e9, 1)
        res[name]["dx_nt_TF"] = round(flop / t_dx / 1e9, 1)
        res[name]["dw_TF"] = round(flop / t_dw / 1e9, 1)
    return res


def attn():
    from paddle_amd.ops import fused as F

    B, H, S, D = 8, 32, 2048, 128
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    do = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    flop_f = 4 * B * H * S * S * D / 2
    out = {}
    t = timeit(lambda: F.flash_attention(q, k, v, causal=True))
    out["pa_fwd_ms"], out["pa_fwd_TF"] = round(t, 3), round(flop_f / t / 1e9, 1)
    o = F.flash_attention(q, k, v, causal=True)

    def pa_bwd():
        torch.autograd.grad(o, (q, k, v), do, retain_graph=True)

    from paddle_amd.ops import _native as N

    variants = [int(x) for x in os.environ.get("PA_FA_BWD_VARIANTS", "1").split(",")]
    for rep in range(2):
        for var in variants:
            N.call("pa_fa_bwd_set_variant", var)
            t = timeit(pa_bwd)
            out[f"pa_bwd_v{var}_ms_r{rep}"] = round(t, 3)
            out[f"pa_bwd_v{var}_TF_r{rep}"] = round(2.5 * flop_f / t / 1e9, 1)
    N.call("pa_fa_bwd_set_variant", 4)
    qt, kt, vt = (x.detach().transpose(1, 2).contiguous().requires_grad_() for x in (q, k, v))
    sd = lambda: torch.nn.functional.scaled_dot_product_attention(qt, kt, vt, is_causal=True)  # noqa: E731
    try:
        t = timeit(sd)
        out["sdpa_fwd_ms"], out["sdpa_fwd_TF"] = round(t, 3), round(flop_f / t / 1e9, 1)
        o2 = sd()
        dot = do.transpose(1, 2).contiguous()
        t = timeit(lambda: torch.autograd.grad(o2, (qt, kt, vt), dot, retain_graph=True))
        out["sdpa_bwd_ms"], out["sdpa_bwd_TF"] = round(t, 3), round(2.5 * flop_f / t / 1e9, 1)
    except Exception as e:  # noqa: BLE001
        out["sdpa_error"] = str(e)[:200]
    return out


if __name__ == "__main__":
    what = sys.argv[1:] or ["gemm", "attn"]
    r = {}
    if "gemm" in what:
        r["gemm"] = gemms()
    if "attn" in what:
        r["attn"] = attn()
    print(json.dumps(r, indent=1))
