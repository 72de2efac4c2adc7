"""Replay of tuned library-GEMM solutions (hipBLASLt / rocBLAS), opt-in.

The training steps of the flagship models do not use it: every LLaMA / GPT / MoE
projection, LM head and expert GEMM runs on the hand-written gfx950 kernel
(csrc/kernels/gemm.hip, ops/gemm.py).  What remains on the vendor library are plain
``torch.matmul`` calls outside those paths (user code, odd shapes the native kernel
does not take).  For those, ``benchmarks/gemm_tune.py`` searches every hipBLASLt
solution once on the MI355X (PyTorch TunableOp) and stores the winners under
``paddle_amd/tuning/gfx950_<model>.csv``; ``enable(model)`` makes later library GEMMs
of those shapes dispatch straight to the stored solution (``bench.py --tuned-gemm``).

The tuning file carries validator lines (PyTorch / ROCm / hipBLASLt versions); a file
from another software stack is rejected by TunableOp and the heuristic pick is used.
"""
from __future__ import annotations

import os

TUNING_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning")


def linear_shapes(model: str) -> dict:
    """{name: (K, N)} of the plain linear GEMMs (y[T,N] = x[T,K] @ W[K,N]) of a model."""
    if model.startswith("llama"):
        from ..models.llama import LLAMA_CONFIGS, LlamaConfig

        c = LlamaConfig(**LLAMA_CONFIGS[model])
        H, I, D = c.hidden_size, c.intermediate_size, c.head_dim
        return {"qkv": (H, (c.num_attention_heads + 2 * c.kv_heads) * D), "o": (H, H),
                "gate_up": (H, 2 * I), "down": (I, H), "lm_head": (H, c.vocab_size)}
    if model.startswith("gpt"):
        from ..models.gpt import GPT_CONFIGS, GPTConfig

        c = GPTConfig(**GPT_CONFIGS[model])
        H = c.hidden_size
        I = getattr(c, "intermediate_size", None) or 4 * H
        return {"qkv": (H, 3 * H), "o": (H, H), "fc1": (H, I), "fc2": (I, H), "lm_head": (H, c.vocab_size)}
    raise KeyError(model)


def tuning_file(model: str) -> str:
    return os.path.join(TUNING_DIR, f"gfx950_{model}.csv")


def enable(model: str, path: str | None = None, verbose: bool = False) -> bool:
    """Load the stored GEMM solutions for ``model`` (no tuning at run time).

    Returns True when a tuning file was found and TunableOp is on."""
    import torch

    p = path or tuning_file(model)
    if not (torch.cuda.is_available() and os.path.exists(p)):
        return False
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(False)
    torch.cuda.tunable.set_filename(p, False)
    ok = torch.cuda.tunable.read_file(p)
    if verbose:
        print(f"[gemm_tuning] {p}: {'loaded' if ok else 'rejected'} "
              f"({len(torch.cuda.tunable.get_results())} solutions)", flush=True)
    if not ok:
        torch.cuda.tunable.enable(False)
    return bool(ok)
