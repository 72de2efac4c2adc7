"""The composed hybrid step runs on the framework's own reverse pass:
with torch.autograd.backward / torch.autograd.grad / Tensor.backward and
torch.utils.checkpoint.checkpoint patched to raise in every rank, the 8-rank gloo
GPT TP2 x PP2 x sharding-3 run still matches the single-process reference (1F1B
micro-batches recorded on per-micro-batch tapes, received activations as watched
tape inputs, ZeRO-3 regather nodes on the tape, vocab-parallel CE / bias / position
nodes with hand-written backwards).  Also: recompute on the tape reproduces the
plain tape gradients.  Reference: python/paddle/fluid/backward.py:315-469 (the
framework differentiates its own programs)."""
import pytest
import torch

from dist_util import run_dist
from hybrid_common import check, reference, worker


def _forbid_torch_autograd():
    def boom(*a, **k):
        raise AssertionError("torch autograd was used")

    torch.autograd.backward = boom
    torch.autograd.grad = boom
    torch.Tensor.backward = boom
    import torch.utils.checkpoint as ckpt

    ckpt.checkpoint = boom


def _strict_worker(rank, world, *args):
    _forbid_torch_autograd()
    return worker(rank, world, *args)


@pytest.mark.timeout(600)
def test_hybrid_tp2_pp2_sharding3_without_torch_autograd():
    ref_losses, init, ref_final = reference(4)
    res = run_dist(_strict_worker, 8, init, 2, 2, 2, "cpu")
    check(res, ref_losses, ref_final, loss_tol=2e-5, atol=2e-5)


@pytest.mark.parametrize("model", ["gpt", "llama"])
def test_recompute_on_tape_matches_plain_tape(model):
    from paddle_amd.autograd import tape
    from paddle_amd.models.gpt import GPT_CONFIGS, GPTConfig, GPTForCausalLM
    from paddle_amd.models.llama import LLAMA_CONFIGS, LlamaConfig, LlamaForCausalLM

    def make(rc):
        torch.manual_seed(0)
        if model == "gpt":
            return GPTForCausalLM(GPTConfig(**{**GPT_CONFIGS["gpt-tiny"], "num_hidden_layers": 2}, dtype="float32",
                                            recompute=rc), "cpu")
        return LlamaForCausalLM(LlamaConfig(**LLAMA_CONFIGS["llama-tiny"], dtype="float32", recompute=rc), "cpu")

    ids = torch.randint(0, 500, (2, 17), generator=torch.Generator().manual_seed(1))
    grads = []
    for rc in (False, True):
        m = make(rc)
        m.train()
        with tape.recording() as t:
            loss = m(ids[:, :-1], ids[:, 1:])
        t.backward(loss)
        grads.append([p.grad.clone() for p in m.parameters()])
    for a, b in zip(*grads):
        assert torch.allclose(a, b, atol=1e-6, rtol=1e-5)
