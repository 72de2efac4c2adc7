"""LLaMA gate|up checkpoint layout: the fused SwiGLU MLP keeps gate|up
interleaved in 16-column blocks IN MEMORY, but state dicts always carry the
canonical [gate | up] matrix, so a checkpoint written as [gate | up] (before the
interleaving existed, or by any other tool) loads into the same function."""
import torch
import torch.nn.functional as F

from paddle_amd import ops
from paddle_amd.models.llama import LLAMA_CONFIGS, LlamaConfig, LlamaForCausalLM


def _model(seed):
    torch.manual_seed(seed)
    cfg = LlamaConfig(**dict(LLAMA_CONFIGS["llama-tiny"], dtype="float32", intermediate_size=704))
    return LlamaForCausalLM(cfg, device="cpu")


def test_state_dict_is_canonical_gate_up():
    m = _model(0)
    layer = m.layers[0]
    assert layer.mlp_interleaved
    sd = m.state_dict()
    g, u = ops.deinterleave_gate_up(layer.gate_up_proj.detach())
    assert torch.equal(sd["layers.0.gate_up_proj"], torch.cat([g, u], -1))
    # the canonical matrix computes the textbook SwiGLU: silu(x W_gate) * (x W_up)
    x = torch.randn(5, m.cfg.hidden_size)
    I = m.cfg.intermediate_size
    w = sd["layers.0.gate_up_proj"]
    want = F.silu(x @ w[:, :I]) * (x @ w[:, I:])
    gg, uu = ops.deinterleave_gate_up(x @ layer.gate_up_proj.detach())
    torch.testing.assert_close(F.silu(gg) * uu, want)


def test_pre_interleave_checkpoint_round_trips_through_load_paths():
    a = _model(0)
    sd = {k: v.clone() for k, v in a.state_dict().items()}  # canonical [gate | up]
    ids = torch.randint(0, a.cfg.vocab_size, (2, 17))
    ref = a(ids[:, :-1], ids[:, 1:]).item()
    for load in ("load_state_dict", "set_state_dict"):
        b = _model(1)
        getattr(b, load)(sd)
        for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
            assert torch.equal(p, q), (load, n)
        assert b(ids[:, :-1], ids[:, 1:]).item() == ref
