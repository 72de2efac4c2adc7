"""ops/accum.py: deferred weight-gradient work is dropped, not leaked, when an
accumulated step is abandoned (ops/grouped.py stash)."""
import pytest
import torch

from paddle_amd.ops import accum


def test_discard_runs_registered_hooks_and_grouped_stash_is_cleared():
    from paddle_amd.ops import grouped as GR

    GR._STASH[123] = ["stale"]
    accum.discard()
    assert not GR._STASH


def test_no_sync_exception_and_zero_grad_discard():
    from paddle_amd.models.llama import LLAMA_CONFIGS, LlamaConfig, LlamaForCausalLM
    from paddle_amd.ops import grouped as GR
    from paddle_amd.parallel.sharding import FlatShardedOptimizer

    torch.manual_seed(0)
    m = LlamaForCausalLM(LlamaConfig(**dict(LLAMA_CONFIGS["llama-tiny"], dtype="float32")), device="cpu")
    opt = FlatShardedOptimizer(m.named_parameters(), lr=1e-3, grad_dtype=torch.float32)
    with pytest.raises(RuntimeError):
        with opt.no_sync():
            assert accum.deferring()
            GR._STASH[1] = ["pending"]
            raise RuntimeError("micro-batch failed")
    assert not accum.deferring() and not GR._STASH
    GR._STASH[2] = ["pending"]
    opt.zero_grad()
    assert not GR._STASH
