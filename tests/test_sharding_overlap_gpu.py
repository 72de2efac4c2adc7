"""The sharded DP engine's GPU overlap machinery (reduce-scatter on the comm stream
during backward, parameter all-gathers issued after AdamW and waited per bucket at
first use in the next forward) on real HIP streams: 2 ranks share the one GPU of
the test box over gloo (RCCL refuses two ranks on one device), bf16 tiny LLaMA,
compared with single-process training on the concatenated batch."""
import pytest
import torch

from dist_util import run_dist

pytestmark = pytest.mark.gpu


def _cfg():
    from paddle_amd.models.llama import LLAMA_CONFIGS, LlamaConfig

    return LlamaConfig(**LLAMA_CONFIGS["llama-tiny"])   # bf16: the fused GPU kernels' dtype


def _batches(n, B=4, S=65, V=512):
    g = torch.Generator().manual_seed(7)
    return [torch.randint(0, V, (B, S), generator=g) for _ in range(n)]


def _train(rank, world, steps, overlap_allgather):
    from paddle_amd.models.llama import LlamaForCausalLM
    from paddle_amd.parallel.sharding import FlatShardedOptimizer

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    m = LlamaForCausalLM(_cfg(), device=dev)
    opt = FlatShardedOptimizer(m.named_parameters(), lr=1e-3, grad_clip=1.0, bucket_mb=1,
                               overlap=True, overlap_allgather=overlap_allgather)
    assert world == 1 or opt.comm_stream is not None
    losses = []
    for b in _batches(steps):
        part = b.chunk(world)[rank].to(dev)
        loss = m(part[:, :-1], part[:, 1:])
        loss.backward()
        opt.step()
        opt.zero_grad()
        losses.append(loss.detach())
    opt.sync_params()
    torch.cuda.synchronize()
    return [x.item() for x in losses], torch.cat([p.detach().reshape(-1).float().cpu() for p in m.parameters()])


def _single(steps):
    import torch.distributed as dist

    return _train(0, 1, steps, False) if not dist.is_initialized() else None


@pytest.mark.parametrize("overlap_allgather", [False, True])
def test_overlapped_sharded_dp_matches_single_process_on_gpu(overlap_allgather):
    steps = 3
    ref_losses, ref_params = _train(0, 1, steps, False)
    res = run_dist(_train, 2, steps, overlap_allgather)
    (l0, p0), (l1, p1) = res
    assert torch.isfinite(p0).all() and torch.isfinite(ref_params).all()
    assert torch.equal(p0, p1)                              # ranks hold identical parameters
    for a, b, r in zip(l0, l1, ref_losses):
        assert abs((a + b) / 2 - r) < 3e-2, (l0, l1, ref_losses)
    # bf16 parameters: DP and single-process differ by reduction order only
    assert ((p0 - ref_params).abs() > 2e-2).float().mean() < 1e-3


def _train_tape(rank, world, steps, accum):
    """bench.py's step: forward on the framework tape (torch autograd off), the
    reverse pass seeded with 1/accum, grad-ready hooks driving the sharded
    optimizer's bucket reduce-scatters, no_sync on all but the last micro-step."""
    from paddle_amd.autograd import tape
    from paddle_amd.models.llama import LlamaForCausalLM
    from paddle_amd.parallel.sharding import FlatShardedOptimizer

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    m = LlamaForCausalLM(_cfg(), device=dev)
    opt = FlatShardedOptimizer(m.named_parameters(), lr=1e-3, grad_clip=1.0, bucket_mb=1, overlap=True,
                               overlap_allgather=True, grad_dtype=torch.float32)
    losses = []
    bs = _batches(steps * accum)
    for s in range(steps):
        tot = 0.0
        for a in range(accum):
            part = bs[s * accum + a].chunk(world)[rank].to(dev)

            def micro():
                with tape.recording() as t:
                    loss = m(part[:, :-1], part[:, 1:])
                t.backward(loss, torch.full_like(loss, 1.0 / accum))
                return loss

            if a < accum - 1:
                with opt.no_sync():
                    loss = micro()
            else:
                loss = micro()
            tot += loss.item() / accum
        opt.step()
        opt.zero_grad()
        losses.append(tot)
    opt.sync_params()
    torch.cuda.synchronize()
    return losses, torch.cat([p.detach().reshape(-1).float().cpu() for p in m.parameters()])


def test_tape_sharded_dp_with_accumulation_matches_single_process_on_gpu():
    """The N>1 bench path (tape + fp32 main_grad + accumulation + overlapped
    reduce-scatter / all-gather) on 2 ranks equals one process on the full batch."""
    steps, accum = 3, 2
    ref_losses, ref_params = _train_tape(0, 1, steps, accum)
    (l0, p0), (l1, p1) = run_dist(_train_tape, 2, steps, accum)
    assert torch.equal(p0, p1)
    for a, b, r in zip(l0, l1, ref_losses):
        assert abs((a + b) / 2 - r) < 3e-2, (l0, l1, ref_losses)
    assert ((p0 - ref_params).abs() > 2e-2).float().mean() < 1e-3
