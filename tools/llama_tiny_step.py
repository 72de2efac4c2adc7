"""A few LLaMA-tiny training steps on the framework tape (for kernel traces and
allocator A/B runs): ``rocprofv3 --kernel-trace --stats -d DIR -- python
tools/llama_tiny_step.py [steps]``.  Prints one JSON line with the per-step losses
and, under FLAGS_allocator_strategy=buddy, the buddy allocator's statistics."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import paddle_amd  # noqa: E402,F401  (installs the allocator selected by FLAGS_allocator_strategy)
from paddle_amd import runtime  # noqa: E402
from paddle_amd.autograd import tape  # noqa: E402
from paddle_amd.models.llama import LLAMA_CONFIGS, LlamaConfig, LlamaForCausalLM  # noqa: E402
from paddle_amd.parallel.sharding import FlatShardedOptimizer  # noqa: E402

torch.manual_seed(0)
cfg = LlamaConfig(**LLAMA_CONFIGS["llama-tiny"])
model = LlamaForCausalLM(cfg, device="cuda")
opt = FlatShardedOptimizer(model.named_parameters(), lr=1e-3, weight_decay=0.1, grad_clip=1.0,
                           grad_dtype=torch.float32)
ids = torch.randint(0, cfg.vocab_size, (4, 257), generator=torch.Generator().manual_seed(1)).cuda()
torch.cuda.synchronize()
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
losses = []
for step in range(steps):
    with tape.recording() as t:
        loss = model(ids[:, :-1], ids[:, 1:])
    t.backward(loss)
    opt.step()
    opt.zero_grad()
    losses.append(float(loss))
torch.cuda.synchronize()
out = {"losses": losses, "allocator": os.environ.get("FLAGS_allocator_strategy", "buddy")}
if out["allocator"] == "buddy" and runtime.available():
    out["buddy"] = runtime.torch_allocator_stats(0)
print(json.dumps(out))
