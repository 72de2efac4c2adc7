"""Overlapped optimizer update (FlatShardedOptimizer, one rank): AdamW runs per
bucket on a side stream, each parameter's first read in the next forward waits
for its own bucket, and the next reverse pass waits for the rest.  Trained with
the framework tape it must give bit-identical losses and parameters to the
single-kernel update, up to the run-to-run nondeterminism of the float-atomic
kernels (split-K GEMM partials, attention dQ) whose addition order depends on timing."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _train(overlap, steps=4):
    from paddle_amd.autograd import tape
    from paddle_amd.models.llama import LLAMA_CONFIGS, LlamaConfig, LlamaForCausalLM
    from paddle_amd.parallel.sharding import FlatShardedOptimizer

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    cfg = LlamaConfig(**LLAMA_CONFIGS["llama-tiny"])
    model = LlamaForCausalLM(cfg, device=dev)
    # small buckets: many side-stream launches and per-bucket waits
    opt = FlatShardedOptimizer(model.named_parameters(), lr=1e-3, grad_dtype=torch.float32, grad_clip=1.0,
                               bucket_mb=1, overlap_update=overlap)
    assert opt.overlap_update == overlap and len(opt.buckets) > 2
    g = torch.Generator().manual_seed(1)
    losses = []
    for i in range(steps):
        ids = torch.randint(0, cfg.vocab_size, (2, 129), generator=g).to(dev)
        for a in range(2):  # two micro-batches: accumulation into main grads
            with tape.recording() as t:
                loss = model(ids[:, :-1], ids[:, 1:])
            t.backward(loss, torch.full_like(loss, 0.5))
        opt.step()
        opt.zero_grad()
        losses.append(loss.item())
    opt.sync_params()
    torch.cuda.synchronize()
    return losses, torch.cat([p.detach().float().reshape(-1) for p in model.parameters()])


def test_overlapped_update_matches_single_kernel_update():
    la, pa = _train(True)
    lb, pb = _train(False)
    assert la[0] == lb[0]  # before any update: same model, same data
    for a, b in zip(la, lb):
        assert abs(a - b) < 1e-3 * abs(b), (la, lb)
    assert (pa - pb).abs().max().item() < 1e-3, (pa - pb).abs().max().item()
    # both runs moved the parameters by the same amounts (a stale read of a
    # parameter would show as a whole missed update: lr-sized errors)
    lc, pc = _train(False)
    assert (pa - pb).abs().max() <= 4 * (pc - pb).abs().max() + 1e-5
