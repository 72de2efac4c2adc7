"""LLaMA + flat sharded DP engine on CPU (gloo), in the spirit of the reference's
parallel_executor_test_base.check_network_convergence
(python/paddle/fluid/tests/unittests/parallel_executor_test_base.py:29):
the same model trained data-parallel on 2 ranks must match single-process
training on the concatenated batch."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from paddle_amd.models.llama import LLAMA_CONFIGS, LlamaConfig, LlamaForCausalLM
from paddle_amd.parallel.sharding import FlatShardedOptimizer

from dist_util import assert_adam_close, run_dist


def _cfg():
    return LlamaConfig(**LLAMA_CONFIGS["llama-tiny"], dtype="float32")


def _batches(n, B=4, S=33, V=512):
    g = torch.Generator().manual_seed(7)
    return [torch.randint(0, V, (B, S), generator=g) for _ in range(n)]


def _train_single(steps):
    torch.manual_seed(0)
    m = LlamaForCausalLM(_cfg(), device="cpu")
    opt = FlatShardedOptimizer(m.named_parameters(), lr=1e-3, grad_clip=1.0, bucket_mb=1)
    losses = []
    for b in _batches(steps):
        loss = m(b[:, :-1], b[:, 1:])
        loss.backward()
        opt.step()
        opt.zero_grad()
        losses.append(loss.item())
    return losses, torch.cat([p.detach().reshape(-1) for p in m.parameters()])


def _worker(rank, world, steps, overlap_allgather=False):
    torch.manual_seed(0)
    m = LlamaForCausalLM(_cfg(), device="cpu")
    opt = FlatShardedOptimizer(m.named_parameters(), lr=1e-3, grad_clip=1.0, bucket_mb=1,
                               overlap_allgather=overlap_allgather)
    assert len(opt.buckets) > 1
    losses = []
    for b in _batches(steps):
        part = b.chunk(world)[rank]
        loss = m(part[:, :-1], part[:, 1:])
        loss.backward()
        opt.step()
        opt.zero_grad()
        if overlap_allgather:
            # gathers are deferred to first use in the next forward
            assert all(getattr(p, "_pa_pending", None) is not None for p in m.parameters())
        t = torch.tensor([loss.item()])
        torch.distributed.all_reduce(t)
        losses.append(t.item() / world)
    opt.sync_params()
    return losses, torch.cat([p.detach().reshape(-1) for p in m.parameters()])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_tiny_llama_cpu_converges():
    losses, _ = _train_single(15)
    assert losses[-1] < losses[0]


@pytest.mark.parametrize("overlap_allgather", [False, True])
def test_sharded_dp_matches_single_process(overlap_allgather):
    steps = 4
    ref_losses, ref_params = _train_single(steps)
    losses, params = run_dist(_worker, 2, steps, overlap_allgather)[0]
    for a, b in zip(losses, ref_losses):
        assert abs(a - b) < 1e-4, (losses, ref_losses)
    assert_adam_close(params, ref_params, atol=1e-5, rtol=1e-4, lr=1e-3, steps=steps)


def _worker_accum(rank, world, steps, accum):
    # Fleet accumulate_steps: `accum` micro-batches per optimizer step, the first
    # accum-1 under no_sync (no reduce-scatter), the last one syncing the sum
    torch.manual_seed(0)
    m = LlamaForCausalLM(_cfg(), device="cpu")
    opt = FlatShardedOptimizer(m.named_parameters(), lr=1e-3, grad_clip=1.0, bucket_mb=1)
    for b in _batches(steps):
        mbs = b.chunk(world)[rank].chunk(accum)
        for i, mb in enumerate(mbs):
            if i < accum - 1:
                with opt.no_sync():
                    (m(mb[:, :-1], mb[:, 1:]) / accum).backward()
            else:
                (m(mb[:, :-1], mb[:, 1:]) / accum).backward()
        opt.step()
        opt.zero_grad()
    opt.sync_params()
    return torch.cat([p.detach().reshape(-1) for p in m.parameters()])


@pytest.mark.parametrize("world", [1, 2])
def test_grad_accumulation_matches_full_batch(world):
    steps = 3
    _, ref_params = _train_single(steps)
    if world == 1:
        params = _worker_accum(0, 1, steps, 2)
    else:
        params = run_dist(_worker_accum, 2, steps, 2)[0]
    assert_adam_close(params, ref_params, atol=1e-5, rtol=1e-4, lr=1e-3, steps=steps)
