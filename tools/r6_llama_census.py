#!/usr/bin/env python3
"""Steady-state kernel census of the LLaMA-7B bench step: the
bench model / optimizer / data exactly as bench.py builds them, warmup steps run
unrestricted, then ONE full step (2 micro-batches, tape backward, sharded AdamW) runs
inside a strict-native region (FLAGS_strict_native=1): any ATen device kernel in the
timed step raises.  Prints one JSON line with the step's native-op census."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from paddle_amd.autograd import tape  # noqa: E402
from paddle_amd.models.llama import LLAMA_CONFIGS, LlamaConfig, LlamaForCausalLM  # noqa: E402
from paddle_amd.parallel.sharding import FlatShardedOptimizer  # noqa: E402
from paddle_amd.utils import strict  # noqa: E402

model_name = sys.argv[1] if len(sys.argv) > 1 else "llama-7b"
warm = int(sys.argv[2]) if len(sys.argv) > 2 else 2
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
torch.manual_seed(1234)
cfg = LlamaConfig(**dict(LLAMA_CONFIGS[model_name], max_position_embeddings=2048))
model = LlamaForCausalLM(cfg, device=dev)
opt = FlatShardedOptimizer(model.named_parameters(), lr=3e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1,
                           grad_clip=1.0, bucket_mb=256, overlap=True, overlap_allgather=True, overlap_update=True,
                           grad_dtype=torch.float32)
mb, S, accum = 8, 2048, 2
gen = torch.Generator().manual_seed(42)
pool = [torch.randint(0, cfg.vocab_size, (mb, S + 1), generator=gen).to(dev) for _ in range(4)]


def step(i):
    for a in range(accum):
        b = pool[(i * accum + a) % len(pool)]
        ctx = opt.no_sync() if a < accum - 1 else __import__("contextlib").nullcontext()
        with ctx:
            with tape.recording() as t:
                loss = model(b[:, :-1], b[:, 1:])
            t.backward(loss, torch.full_like(loss, 1.0 / accum))
    opt.step()
    opt.zero_grad()
    return loss


for i in range(warm):
    step(i)
torch.cuda.synchronize()
os.environ["FLAGS_strict_native"] = "1"  # the steady-state step only: any ATen device kernel raises
strict.reset()
with strict.region("llama7b:steady_step"):
    loss = step(warm)
torch.cuda.synchronize()
rep = strict.report()
print(json.dumps({"model": model_name, "warmup_steps": warm, "loss": float(loss),
                  "aten_kernels": rep["aten_kernels"], "fallbacks": rep["fallbacks"],
                  "native_ops": dict(sorted(rep["native_ops"].items(), key=lambda kv: -kv[1])[:40])
                  if isinstance(rep.get("native_ops"), dict) else rep.get("native_ops")}))
