"""Minimal driver for rocprofv3 counter passes over pa_gemm: runs one form of one
LLaMA-7B GEMM `reps` times (random-normal operands).
usage: gemm_prof.py {fwd,dx,dw} {qkv,o,gate_up,down,lm_head} [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_amd.ops import gemm as G  # noqa: E402

SHAPES = {"qkv": (4096, 12288), "o": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096),
          "lm_head": (4096, 32000)}
form, name = sys.argv[1], sys.argv[2]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
K, Nn = SHAPES[name]
T = 16384
x = torch.randn(T, K, device="cuda").to(torch.bfloat16)
w = (torch.randn(K, Nn, device="cuda") * 0.02).to(torch.bfloat16)
dy = torch.randn(T, Nn, device="cuda").to(torch.bfloat16)
mg = torch.zeros(K, Nn, device="cuda")
for _ in range(reps):
    if form == "fwd":
        G.linear_fwd(x, w)
    elif form == "dx":
        G.linear_dx(dy, w)
    else:
        G.linear_dw(x, dy, out=mg, accumulate=True)
torch.cuda.synchronize()
print("done", form, name, reps)
