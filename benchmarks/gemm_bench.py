"""pa_gemm (hand-written gfx950 MFMA) vs torch.matmul (hipBLASLt) on the LLaMA-7B
training GEMMs (M = 16384 tokens), interleaved in one process (guide §5.4 rule 24),
random-normal operands.  Prints one JSON line per (shape, form)."""
import json
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from paddle_amd.ops import gemm as G  # noqa: E402

T = 16384
SHAPES = {"qkv": (4096, 12288), "o": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096),
          "lm_head": (4096, 32000)}


def timeit(fn, reps):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps


def main():
    forms = sys.argv[1].split(",") if len(sys.argv) > 1 else ["fwd", "dx", "dw"]
    names = sys.argv[2].split(",") if len(sys.argv) > 2 else list(SHAPES)
    rounds = 5
    for name in names:
        K, Nn = SHAPES[name]
        x = torch.randn(T, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(K, Nn, device="cuda") * 0.02).to(torch.bfloat16)
        dy = torch.randn(T, Nn, device="cuda").to(torch.bfloat16)
        mg = torch.zeros(K, Nn, device="cuda")
        for form in forms:
            flops = 2.0 * T * K * Nn
            if form == "fwd":
                ours, ref = (lambda: G.linear_fwd(x, w)), (lambda: torch.matmul(x, w))
            elif form == "dx":
                ours, ref = (lambda: G.linear_dx(dy, w)), (lambda: torch.matmul(dy, w.t()))
            else:
                ours = lambda: G.linear_dw(x, dy, out=mg, accumulate=True)  # noqa: E731
                ref = lambda: mg.add_(torch.mm(x.t(), dy, out_dtype=torch.float32))  # noqa: E731
            for f in (ours, ref):
                f()
            torch.cuda.synchronize()
            to, tr = [], []
            for _ in range(rounds):
                to.append(timeit(ours, 5))
                tr.append(timeit(ref, 5))
            to.sort(), tr.sort()
            rec = {"shape": name, "form": form, "M": T, "K": K, "N": Nn,
                   "pa_ms": round(to[len(to) // 2], 4), "torch_ms": round(tr[len(tr) // 2], 4),
                   "pa_tflops": round(flops / to[len(to) // 2] / 1e9, 1),
                   "torch_tflops": round(flops / tr[len(tr) // 2] / 1e9, 1)}
            rec["ratio"] = round(rec["torch_ms"] / rec["pa_ms"], 3)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
