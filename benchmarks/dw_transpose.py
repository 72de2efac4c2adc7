#!/usr/bin/env python3
"""Does re-laying the dW GEMM operands token-inner pay on gfx950?

For each LLaMA-7B linear at 16384 tokens: hipBLASLt dW in the TN form
(x^T dY, beta=1 into a bf16 main grad) vs our HIP transpose of x and dY + the NT
form; plus transpose bandwidth (ours vs torch's strided copy) and the forward
NN (x W) vs NT (x (W^T)^T) with a transposed weight copy.  Median of interleaved
repetitions in one process."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle_amd.ops import fused as F  # noqa: E402


def timeit(fn, reps=15, warm=3):
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


def main():
    T = 16384
    shapes = {"qkv": (4096, 12288), "o": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096),
              "lm_head": (4096, 32000)}
    tot = {"tn": 0.0, "tr_nt": 0.0, "trx_nn": 0.0, "fwd_nn": 0.0, "fwd_nt": 0.0}
    for name, (K, N) in shapes.items():
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(K, N, device="cuda", dtype=torch.bfloat16) * 0.02
        wt = F.transpose2d(w)
        g = torch.zeros(K, N, device="cuda", dtype=torch.bfloat16)
        r = {}
        r["dw_tn_ms"] = timeit(lambda: g.addmm_(x.t(), dy))
        r["dw_tr_nt_ms"] = timeit(lambda: g.addmm_(F.transpose2d(x), F.transpose2d(dy).t()))
        xt, dyt = F.transpose2d(x), F.transpose2d(dy)
        r["dw_nt_only_ms"] = timeit(lambda: g.addmm_(xt, dyt.t()))
        r["dw_trx_nn_ms"] = timeit(lambda: g.addmm_(F.transpose2d(x), dy))
        r["dw_nn_only_ms"] = timeit(lambda: g.addmm_(xt, dy))
        r["tr_x_ms"] = timeit(lambda: F.transpose2d(x))
        r["tr_x_torch_ms"] = timeit(lambda: x.t().contiguous())
        r["tr_x_TBps"] = 2 * x.numel() * 2 / r["tr_x_ms"] / 1e9
        r["tr_dy_ms"] = timeit(lambda: F.transpose2d(dy))
        r["fwd_nn_ms"] = timeit(lambda: torch.matmul(x, w))
        r["fwd_nt_ms"] = timeit(lambda: torch.matmul(x, wt.t()))
        ok = torch.allclose(F.transpose2d(x), x.t())
        r = {k: round(v, 4) for k, v in r.items()}
        r["transpose_exact"] = bool(ok)
        tot["tn"] += r["dw_tn_ms"]
        tot["tr_nt"] += r["dw_tr_nt_ms"]
        tot["trx_nn"] += r["dw_trx_nn_ms"]
        tot["fwd_nn"] += r["fwd_nn_ms"]
        tot["fwd_nt"] += r["fwd_nt_ms"]
        print(json.dumps({"shape": name, "K": K, "N": N, **r}), flush=True)
    print(json.dumps({"summary": {k: round(v, 3) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
