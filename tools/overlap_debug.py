"""Debug: overlapped optimizer update vs single-kernel update on llama-tiny --
per-parameter max |master diff| after each step, with and without a full sync
right after step()."""
import sys

import torch

sys.path.insert(0, ".")
from paddle_amd.autograd import tape  # noqa: E402
from paddle_amd.models.llama import LLAMA_CONFIGS, LlamaConfig, LlamaForCausalLM  # noqa: E402
from paddle_amd.parallel.sharding import FlatShardedOptimizer  # noqa: E402

dev = torch.device("cuda", 0)


def run(overlap, sync_after, steps=4):
    torch.manual_seed(0)
    cfg = LlamaConfig(**LLAMA_CONFIGS["llama-tiny"])
    model = LlamaForCausalLM(cfg, device=dev)
    opt = FlatShardedOptimizer(model.named_parameters(), lr=1e-3, grad_dtype=torch.float32, grad_clip=1.0,
                               bucket_mb=1, overlap_update=overlap)
    g = torch.Generator().manual_seed(1)
    snaps = []
    for i in range(steps):
        ids = torch.randperm(cfg.vocab_size, generator=g)[:2 * 129].view(2, 129).to(dev)
        for a in range(2):
            with tape.recording() as t:
                loss = model(ids[:, :-1], ids[:, 1:])
            t.backward(loss, torch.full_like(loss, 0.5))
        opt.step()
        if sync_after:
            opt.sync_params()
        opt.zero_grad()
        opt.sync_params()
        torch.cuda.synchronize()
        snaps.append((loss.item(), opt.master.clone()))
    return snaps, opt


ref, opt = run(False, False)
for name, ov, sy in (("ref2", False, False), ("overlap", True, False), ("overlap+sync", True, True)):
    s, _ = run(ov, sy)
    for i, ((la, ma), (lb, mb)) in enumerate(zip(s, ref)):
        d = (ma - mb).abs()
        worst = []
        for n, p, o in zip(opt.names, opt.params, opt.offsets):
            worst.append((d[o:o + p.numel()].max().item(), n))
        worst.sort(reverse=True)
        print(name, "step", i, "loss", la, lb, "max", d.max().item(), "worst", worst[:3], flush=True)
