#!/usr/bin/env python3
"""BatchNorm apply (y = relu(x * s + t)) variants at ResNet-50 bs-256 shapes, one
process per variant (the launcher reads PA_BN_APPLY once), against a device copy of
the same bytes (torch clone) as the achievable-bandwidth reference.
usage: bn_apply_ab.py -> one JSON line per (variant, shape)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import json, sys, torch
sys.path.insert(0, %r)
from paddle_amd.ops import _native as N
res = []
for rows, C in ((256 * 112 * 112, 64), (256 * 56 * 56, 256), (256 * 28 * 28, 512), (256 * 7 * 7, 2048)):
    x = torch.randn(rows, C, device="cuda", dtype=torch.bfloat16)
    y = torch.empty_like(x)
    mean = torch.randn(C, device="cuda"); rstd = torch.rand(C, device="cuda") + 0.5
    w = torch.rand(C, device="cuda"); b = torch.randn(C, device="cuda")
    def run():
        N.call("pa_bn_apply", N.ptr(x), N.ptr(y), N.ptr(mean), N.ptr(rstd), N.ptr(w), N.ptr(b), 0, rows, C, 1,
               N.stream())
    def clone():
        y.copy_(x)
    out = {"rows": rows, "C": C}
    for name, fn in (("bn_apply", run), ("copy", clone)):
        for _ in range(3): fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20): fn()
        e.record(); torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 20
        out[name + "_us"] = round(ms * 1000, 1)
        out[name + "_TBps"] = round(2 * x.numel() * 2 / ms / 1e9, 2)
    ref = torch.relu(x.float() * (rstd * w) + (b - mean * rstd * w)).to(torch.bfloat16)
    run(); torch.cuda.synchronize()
    out["maxerr"] = float((y.float() - ref.float()).abs().max())
    res.append(out)
print(json.dumps(res))
""" % ROOT

for v in ("0", "1", "2", "3"):
    e = dict(os.environ, PA_BN_APPLY=v)
    r = subprocess.run([sys.executable, "-c", CHILD], env=e, capture_output=True, text=True, timeout=300)
    line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-500:]
    print(json.dumps({"variant": v, "res": json.loads(line) if line.startswith("[") else line}), flush=True)
