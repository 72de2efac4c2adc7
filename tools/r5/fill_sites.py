"""Which framework lines issue large ATen fills / zeroings on device tensors during an
ERNIE-MoE training step (the FillFunctor<float> kernels of profiles/r5_moe_fp8_prof.md that
run outside any framework region): wraps torch.zeros / zeros_like / full / Tensor.zero_ /
fill_ and prints (file:line, numel, calls)."""
import collections
import os
import sys
import traceback

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch  # noqa: E402

SITES = collections.Counter()
MIN = 1 << 20


def _site():
    for fr in reversed(traceback.extract_stack()[:-2]):
        if "paddle_amd" in fr.filename or "benchmarks" in fr.filename:
            return f"{fr.filename[fr.filename.rfind('paddle_amd') if 'paddle_amd' in fr.filename else fr.filename.rfind('benchmarks'):]}:{fr.lineno}"
    return "?"


def _wrap_factory(name):
    orig = getattr(torch, name)

    def f(*a, **k):
        t = orig(*a, **k)
        if isinstance(t, torch.Tensor) and t.is_cuda and t.numel() >= MIN:
            SITES[(name, _site(), t.numel())] += 1
        return t
    setattr(torch, name, f)


def _wrap_method(name):
    orig = getattr(torch.Tensor, name)

    def f(self, *a, **k):
        if self.is_cuda and self.numel() >= MIN:
            SITES[(name, _site(), self.numel())] += 1
        return orig(self, *a, **k)
    setattr(torch.Tensor, name, f)


for n in ("zeros", "zeros_like", "full", "full_like", "ones"):
    _wrap_factory(n)
for n in ("zero_", "fill_"):
    _wrap_method(n)

from paddle_amd.autograd import tape  # noqa: E402
from paddle_amd.models.ernie_moe import ERNIE_MOE_CONFIGS, ErnieMoEConfig, ErnieMoEForCausalLM  # noqa: E402
from paddle_amd.parallel.sharding import FlatShardedOptimizer  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
cfg = ErnieMoEConfig(**dict(ERNIE_MOE_CONFIGS["ernie-moe-a3b-8l"], num_hidden_layers=2),
                     use_fp8_experts=True, grouped_experts=True)
m = ErnieMoEForCausalLM(cfg, dev)
opt = FlatShardedOptimizer(m.named_parameters(), lr=1e-4, weight_decay=0.1, grad_clip=1.0, bucket_mb=512,
                           grad_dtype=torch.float32)
ids = torch.randint(0, cfg.vocab_size, (8, 2049), device=dev)
for step in range(3):
    if step == 2:
        SITES.clear()
    for mb in range(4):
        ctx = opt.no_sync() if mb < 3 else None
        if ctx:
            ctx.__enter__()
        with tape.recording() as t:
            loss = m(ids[:, :-1], ids[:, 1:])
        t.backward(loss, torch.full_like(loss, 0.25))
        if ctx:
            ctx.__exit__(None, None, None)
    opt.step()
    opt.zero_grad()
torch.cuda.synchronize()
for (name, site, n), c in sorted(SITES.items(), key=lambda kv: -kv[0][2] * kv[1]):
    print(f"{name:10s} {site:60s} numel={n:>12d} calls={c}")
