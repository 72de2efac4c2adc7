"""Overlapped optimizer update (FlatShardedOptimizer, one rank): AdamW runs per
bucket on a side stream, each parameter's first read in the next forward waits
for its own bucket, and the next reverse pass waits for the rest.  Trained with
the framework tape it must give bit-identical losses and parameters to the
single-kernel update up to last-ulp differences (distinct token ids; a large
Adam epsilon keeps those from being amplified into lr-sized steps)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _train(overlap, steps=4, param_dtype_grads=False):
    from paddle_amd.autograd import tape
    from paddle_amd.models.llama import LLAMA_CONFIGS, LlamaConfig, LlamaForCausalLM
    from paddle_amd.parallel.sharding import FlatShardedOptimizer

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    cfg = LlamaConfig(**LLAMA_CONFIGS["llama-tiny"])
    model = LlamaForCausalLM(cfg, device=dev)
    # small buckets: many side-stream launches and per-bucket waits
    # eps = 1e-2: Adam's normalised step no longer turns last-ulp noise in a ~0
    # gradient into a +-lr update (with eps 1e-8 two runs of the SAME path drift
    # apart by ~lr through the embedding rows of the float-atomic backward)
    opt = FlatShardedOptimizer(model.named_parameters(), lr=1e-3, eps=1e-2, grad_dtype=None if param_dtype_grads else torch.float32,
                               grad_clip=1.0, bucket_mb=1, overlap_update=overlap)
    assert opt.overlap_update == overlap and len(opt.buckets) > 2
    g = torch.Generator().manual_seed(1)
    losses = []
    for i in range(steps):
        # distinct token ids: the embedding backward's float atomics never collide,
        # so the whole step is deterministic and the two updates compare bitwise
        ids = torch.randperm(cfg.vocab_size, generator=g)[:2 * 129].view(2, 129).to(dev)
        for a in range(2):  # two micro-batches: accumulation into main grads
            with tape.recording() as t:
                loss = model(ids[:, :-1], ids[:, 1:])
            t.backward(loss, torch.full_like(loss, 0.5))
        opt.step()
        opt.zero_grad()
        losses.append(loss.item())
    opt.sync_params()
    torch.cuda.synchronize()
    return losses, opt.master.detach().clone()


def test_overlapped_update_matches_single_kernel_update():
    la, pa = _train(True)
    lb, pb = _train(False)
    assert la[0] == lb[0]
    for a, b in zip(la, lb):
        # bf16 forward: last-ulp master differences show up as ~1e-5 relative loss noise
        assert abs(a - b) <= 2e-4 * abs(b), (la, lb)
    # a parameter read before its bucket's update landed would leave a whole AdamW
    # step (~lr = 1e-3) of difference; per-bucket vs whole-buffer launches differ
    # in the last ulp only
    assert (pa - pb).abs().max().item() < 1e-4, (pa - pb).abs().max().item()


def test_overlapped_update_param_dtype_grads_eager_zero_grad():
    """Gradients kept in the parameter dtype (no fp32 main grads): zero_grad()
    zero-fills flat_grad on the main stream right after step() -- it must wait for
    the side stream's update, which is still reading those gradients."""
    la, pa = _train(True, param_dtype_grads=True)
    lb, pb = _train(False, param_dtype_grads=True)
    for a, b in zip(la, lb):
        assert abs(a - b) <= 2e-4 * abs(b), (la, lb)
    assert (pa - pb).abs().max().item() < 1e-4, (pa - pb).abs().max().item()
