#!/usr/bin/env python3
"""Tune the library GEMMs of a model's linear layers with PyTorch TunableOp
(hipBLASLt + rocBLAS solution search on gfx950) and write the winning solutions to
a CSV the training entry points load (``paddle_amd.utils.gemm_tuning``).

Plain library GEMMs are the only GEMMs we leave to hipBLASLt (fused GEMM-shaped work
runs in our own MFMA kernels); the default heuristic pick is not always the fastest
solution for the skinny-K / wide-N shapes of a transformer, so we search once per
(shape, layout) and replay the pick.

Usage (on the MI355X box):
    python benchmarks/gemm_tune.py --model llama-7b --tokens 16384 \
        --out paddle_amd/tuning/gfx950_llama-7b.csv
Prints one JSON line per shape: default vs tuned ms and TFLOP/s for fwd (NN),
dX (NT) and dW-accumulate (TN, beta=1).
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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


def model_shapes(model):
    from paddle_amd.utils.gemm_tuning import linear_shapes

    return linear_shapes(model)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-7b")
    ap.add_argument("--tokens", type=int, nargs="+", default=[16384])
    ap.add_argument("--out", default=None)
    ap.add_argument("--max-ms", type=int, default=15, help="TunableOp time budget per solution")
    args = ap.parse_args()
    out = args.out or os.path.join("paddle_amd", "tuning", f"gfx950_{args.model}.csv")
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    dev = "cuda"
    shapes = model_shapes(args.model)
    cases = []
    for T in args.tokens:
        for name, (K, N) in shapes.items():
            x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
            w = torch.randn(K, N, device=dev, dtype=torch.bfloat16) * 0.02
            dy = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
            g = torch.zeros(K, N, device=dev, dtype=torch.bfloat16)
            cases.append((f"{name}@{T}", 2.0 * T * K * N, {
                "fwd": lambda x=x, w=w: torch.matmul(x, w),
                "dx": lambda dy=dy, w=w: torch.matmul(dy, w.t()),
                "dw": lambda g=g, x=x, dy=dy: g.addmm_(x.t(), dy),
            }))
    # default hipBLASLt heuristic
    res = {}
    for name, flop, fns in cases:
        res[name] = {f"{k}_default_ms": round(timeit(f), 4) for k, f in fns.items()}
    # tuned
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(True)
    torch.cuda.tunable.set_max_tuning_duration(args.max_ms)
    torch.cuda.tunable.set_max_tuning_iterations(40)
    torch.cuda.tunable.set_filename(out, False)
    t0 = time.time()
    for name, flop, fns in cases:
        for k, f in fns.items():
            f()  # first call runs the search
            torch.cuda.synchronize()
        print(f"[tune] {name} searched ({time.time()-t0:.0f}s)", file=sys.stderr, flush=True)
    torch.cuda.tunable.tuning_enable(False)
    for name, flop, fns in cases:
        for k, f in fns.items():
            t = timeit(f)
            r = res[name]
            r[f"{k}_tuned_ms"] = round(t, 4)
            r[f"{k}_default_TF"] = round(flop / r[f"{k}_default_ms"] / 1e9, 1)
            r[f"{k}_tuned_TF"] = round(flop / t / 1e9, 1)
        print(json.dumps({"shape": name, **res[name]}), flush=True)
    # TunableOp writes the results file itself at process exit
    tot_d = sum(v for r in res.values() for k, v in r.items() if k.endswith("default_ms"))
    tot_t = sum(v for r in res.values() for k, v in r.items() if k.endswith("tuned_ms"))
    print(json.dumps({"summary": True, "default_ms": round(tot_d, 3), "tuned_ms": round(tot_t, 3),
                      "speedup": round(tot_d / tot_t, 4), "file": out}), flush=True)


if __name__ == "__main__":
    main()
