#!/usr/bin/env python3
"""Tile-count tail on GPT-3 13B's narrow-output GEMMs (N = 5120 at M = 4096 tokens:
320 256x256 tiles = 1.25 waves on 256 CUs): plain GEMM vs split-K with float
atomics into an fp32 buffer (+ the bf16 cast that would follow).  One JSON line
per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from paddle_amd.ops import gemm as G  # noqa: E402


def bench(fn, iters=20):
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


def main():
    M = 4096
    for name, N, K, form in [("out_fwd", 5120, 5120, "fwd"), ("fc2_fwd", 5120, 20480, "fwd"),
                             ("qkv_dx", 5120, 15360, "dx"), ("fc1_dx", 5120, 20480, "dx"),
                             ("llama_o_fwd_ref", 4096, 4096, "fwd")]:
        Mx = 16384 if name.startswith("llama") else M
        a = torch.randn(Mx, K, device="cuda").to(torch.bfloat16)
        w = torch.randn(K, N, device="cuda").to(torch.bfloat16) if form == "fwd" else \
            torch.randn(N, K, device="cuda").to(torch.bfloat16)
        bk = form == "dx"
        base = bench(lambda: G.gemm(a, w, Mx, N, K, a_kmaj=True, b_kmaj=bk))
        out = torch.empty(Mx, N, dtype=torch.float32, device="cuda")
        res = {"shape": name, "M": Mx, "N": N, "K": K, "plain_ms": round(base, 4),
               "tflops_plain": round(2 * Mx * N * K / base / 1e9, 1)}
        for S in (2, 3, 4):
            tiles = ((Mx + 255) // 256) * ((N + 255) // 256)
            t = bench(lambda: G.gemm_splitk(a, w, Mx, N, K, a_kmaj=True, b_kmaj=bk, out=out,
                                           target_blocks=tiles * S))
            tc = bench(lambda: out.to(torch.bfloat16))
            res[f"splitk{S}_ms"] = round(t, 4)
            res[f"splitk{S}_plus_cast_ms"] = round(t + tc, 4)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
