"""AdamW streaming bandwidth on the flat fp32 master / fp32 moments / fp32 grad /
bf16 model-copy layout of the sharded LLaMA step (ops/optim.py adamw_flat).
Mode: env PA_ADAMW_MODE (0 4-wide, 1 8-wide, 2 8-wide non-temporal).  Prints JSON:
effective TB/s at 30 B/element, plus a correctness check of an odd-sized (tail) case
against the CPU formula."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_amd.ops.optim import adamw_flat  # noqa: E402


def check():
    n = 1000003
    torch.manual_seed(0)
    p = torch.randn(n, device="cuda")
    g = torch.randn(n, device="cuda")
    m = torch.randn(n, device="cuda") * 0.1
    v = torch.rand(n, device="cuda") * 0.1
    out = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    ref = [t.cpu().clone() for t in (p, g, m, v)]
    adamw_flat(p, g, m, v, lr=1e-3, weight_decay=0.1, step=3, param_out=out, decay_end=n // 2)
    rp, rg, rm, rv = ref
    adamw_flat(rp, rg, rm, rv, lr=1e-3, weight_decay=0.1, step=3, decay_end=n // 2)
    torch.cuda.synchronize()
    return max(float((p.cpu() - rp).abs().max()), float((m.cpu() - rm).abs().max()),
               float((v.cpu() - rv).abs().max()), float((out.float().cpu() - rp.bfloat16().float()).abs().max()))


def main():
    n = int(os.environ.get("N", 1_000_000_000))
    p = torch.zeros(n, device="cuda")
    g = torch.full((n,), 1e-3, device="cuda")
    m = torch.zeros(n, device="cuda")
    v = torch.zeros(n, device="cuda")
    out = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    for _ in range(2):
        adamw_flat(p, g, m, v, lr=1e-4, weight_decay=0.1, step=1, param_out=out)
    torch.cuda.synchronize()
    ts = []
    for it in range(5):
        t0 = time.perf_counter()
        adamw_flat(p, g, m, v, lr=1e-4, weight_decay=0.1, step=2 + it, param_out=out)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    best = min(ts)
    print(json.dumps({"mode": os.environ.get("PA_ADAMW_MODE", "2"), "n": n, "ms": round(best * 1e3, 3),
                      "TBps": round(30 * n / best / 1e12, 3), "maxerr": check()}))


if __name__ == "__main__":
    main()
