#!/usr/bin/env python3
"""RMSNorm backward variants at the LLaMA-7B step shape ([16384, 4096] bf16, fused
residual gradient): one process per variant (the launcher reads its knobs once).
usage: norm_bwd_ab.py  -> prints one JSON line per variant."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, sys, torch
sys.path.insert(0, %r)
from paddle_amd.ops import _native as N
T, H, RMS = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
dy = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
h = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
dres = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
w = torch.rand(H, device="cuda", dtype=torch.bfloat16)
rstd = torch.rand(T, device="cuda") + 0.5
dx = torch.empty_like(h); dw = torch.empty_like(w)
ws = torch.empty(2 * 1024 * H, device="cuda")
mean = torch.randn(T, device="cuda")
b = torch.rand(H, device="cuda", dtype=torch.bfloat16)
db = torch.empty_like(w)
def run():
    N.call("pa_norm_bwd", 1, RMS, N.ptr(dy), N.ptr(h), N.ptr(w), None if RMS else N.ptr(mean), N.ptr(rstd),
           N.ptr(dres), N.ptr(dx), N.ptr(dw), None if RMS else N.ptr(db), N.ptr(ws), T, H, N.stream())
for _ in range(5): run()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(50): run()
e.record(); torch.cuda.synchronize()
ms = s.elapsed_time(e) / 50
ref = dx.float()
print(json.dumps({"ms": round(ms, 4), "TBps": round(4 * T * H * 2 / ms / 1e9, 2),
                  "dx_sum": float(ref.double().sum()), "dw_sum": float(dw.double().sum())}))
""" % ROOT

SHAPES = [(16384, 4096, 1), (4096, 5120, 0)]  # LLaMA-7B RMSNorm, GPT-3 13B LayerNorm (mb 2)
for T_, H_, rms in SHAPES:
    for name, env in (("rpb4_g512", {"PA_NORM_BWD_RPB": "4"}), ("rpb16", {"PA_NORM_BWD_RPB": "16"}),
                      ("rpb32", {"PA_NORM_BWD_RPB": "32"}), ("rpb64", {"PA_NORM_BWD_RPB": "64"})):
        e = dict(os.environ, **env)
        out = subprocess.run([sys.executable, "-c", CHILD, str(T_), str(H_), str(rms)], env=e, capture_output=True,
                             text=True, timeout=300)
        line = out.stdout.strip().splitlines()[-1] if out.stdout.strip() else out.stderr[-500:]
        print(json.dumps({"shape": [T_, H_, rms], "variant": name,
                          **(json.loads(line) if line.startswith("{") else {"error": line})}), flush=True)
