#!/usr/bin/env python3
"""Where does a batch-32, hidden-512 LSTM train step spend its time on MI355X?
(stacked_lstm row of the reference suite).  fwd+bwd per batch for: MIOpen packed /
padded in fp32 and bf16, and a step loop (one input-projection GEMM + per-step
recurrent GEMM + pointwise)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

def timeit(fn, n=5, w=2):
    for _ in range(w):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


def main():
    dev = torch.device("cuda")
    B, H = 32, 512
    rng = np.random.RandomState(0)
    lens = torch.from_numpy(np.clip(rng.lognormal(5.25, 0.65, B), 10, 1499).astype(np.int64))
    T = int(lens.max())
    res = {"T": T, "avg_len": float(lens.float().mean())}
    for dt in (torch.float32, torch.bfloat16):
        lstm = torch.nn.LSTM(H, H, batch_first=True).to(dev, dt)
        x = torch.randn(B, T, H, device=dev, dtype=dt, requires_grad=True)

        def packed():
            p = torch.nn.utils.rnn.pack_padded_sequence(x, lens, batch_first=True, enforce_sorted=False)
            _, (h, _) = lstm(p)
            h.float().sum().backward()

        def padded():
            o, _ = lstm(x)
            o.float().sum().backward()

        name = "fp32" if dt == torch.float32 else "bf16"
        try:
            res[f"miopen_packed_{name}_ms"] = round(timeit(packed), 2)
        except Exception as e:  # noqa: BLE001
            res[f"miopen_packed_{name}_ms"] = str(e)[:80]
        try:
            res[f"miopen_padded_{name}_ms"] = round(timeit(padded), 2)
        except Exception as e:  # noqa: BLE001
            res[f"miopen_padded_{name}_ms"] = str(e)[:80]

        wih = torch.randn(H, 4 * H, device=dev, dtype=dt, requires_grad=True)
        whh = torch.randn(H, 4 * H, device=dev, dtype=dt, requires_grad=True)

        def loop():
            xp = (x.reshape(-1, H) @ wih).view(B, T, 4 * H)
            h = torch.zeros(B, H, device=dev, dtype=dt)
            c = torch.zeros(B, H, device=dev, dtype=dt)
            for t in range(T):
                g = xp[:, t] + h @ whh
                i, f, gg, o = g.chunk(4, 1)
                c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
                h = torch.sigmoid(o) * torch.tanh(c)
            h.float().sum().backward()

        res[f"torch_loop_{name}_ms"] = round(timeit(loop, n=2, w=1), 2)

        from paddle_amd.ops import rnn

        xt = x.detach().transpose(0, 1).contiguous().requires_grad_()
        b = torch.zeros(4 * H, device=dev, dtype=dt, requires_grad=True)

        def persistent():
            hs, h, _ = rnn.lstm(xt, wih, whh, b, lens=lens)
            h.float().sum().backward()

        res[f"persistent_{name}_ms"] = round(timeit(persistent), 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
