"""FLAGS_strict_native=1 on the model paths: one training step of
LLaMA-tiny, GPT-tiny (50,257-wide tied LM head on the padded native GEMM) and
ERNIE-MoE-tiny (native routing / router backward) -- forward on the framework tape,
tape backward, flat sharded AdamW -- runs inside one framework region with every
ATen device kernel refused (utils/strict.py raises StrictNativeError), and the Fluid
ResNet program runs on the C++ executor with no Python-kernel or host fallback."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def strict_on():
    old = os.environ.get("FLAGS_strict_native")
    os.environ["FLAGS_strict_native"] = "1"
    try:
        yield
    finally:
        if old is None:
            os.environ.pop("FLAGS_strict_native", None)
        else:
            os.environ["FLAGS_strict_native"] = old


def _model(name):
    dev = torch.device("cuda", 0)
    if name == "llama":
        from paddle_amd.models.llama import LLAMA_CONFIGS, LlamaConfig, LlamaForCausalLM

        cfg = LlamaConfig(**dict(LLAMA_CONFIGS["llama-tiny"], hidden_size=512, intermediate_size=1024,
                                 num_attention_heads=4, max_position_embeddings=2048))
        return LlamaForCausalLM(cfg, dev), cfg.vocab_size
    if name == "gpt":
        from paddle_amd.models.gpt import GPT_CONFIGS, GPTConfig, GPTForCausalLM

        cfg = GPTConfig(**dict(GPT_CONFIGS["gpt-tiny"], vocab_size=50257, max_position_embeddings=2048))
        return GPTForCausalLM(cfg, dev), cfg.vocab_size
    from paddle_amd.models.ernie_moe import ERNIE_MOE_CONFIGS, ErnieMoEConfig, ErnieMoEForCausalLM

    cfg = ErnieMoEConfig(**dict(ERNIE_MOE_CONFIGS["ernie-moe-tiny"], hidden_size=256, moe_intermediate_size=128,
                                intermediate_size=512, grouped_experts=True, max_position_embeddings=2048))
    return ErnieMoEForCausalLM(cfg, dev), cfg.vocab_size


def _steps(name, strict_mode):
    """Three training steps from seed 0; returns (losses, strict report)."""
    from paddle_amd.autograd import tape
    from paddle_amd.parallel.sharding import FlatShardedOptimizer
    from paddle_amd.utils import strict

    torch.manual_seed(0)
    m, V = _model(name)
    opt = FlatShardedOptimizer(m.named_parameters(), lr=1e-4, grad_dtype=torch.float32)
    # 2 x 1024 tokens: the fused GEMM-epilogue paths of the production shapes (the
    # W^T-cached K-major forms need >= 1024 tokens)
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(0, V, (2, 1025), generator=g).cuda()
    losses = []
    strict.reset()
    for _ in range(3):
        with strict.region(f"{name}:step") if strict_mode else __import__("contextlib").nullcontext():
            with tape.recording() as t:
                loss = m(ids[:, :-1], ids[:, 1:])
            t.backward(loss)
            opt.step()
            opt.zero_grad()
        losses.append(float(loss))
    torch.cuda.synchronize()
    return losses, strict.report()


@pytest.mark.parametrize("name", ["llama", "gpt", "ernie"])
def test_model_training_step_under_strict_native(name, monkeypatch):
    """The strict run refuses every ATen kernel AND trains along the same loss
    trajectory as the unrestricted run of the same seeds (not just finite losses)."""
    monkeypatch.delenv("FLAGS_strict_native", raising=False)
    free, _ = _steps(name, False)
    monkeypatch.setenv("FLAGS_strict_native", "1")
    losses, rep = _steps(name, True)
    assert rep["aten_kernels"] == {} and rep["fallbacks"] == {}, rep
    assert all(np.isfinite(losses)), losses
    np.testing.assert_allclose(losses, free, rtol=2e-3, atol=1e-4)


def test_fluid_resnet_native_engine_under_strict_native(strict_on):
    import paddle_amd.fluid as fluid
    from native_engine_cases import train

    _, _, _, exe = train("resnet_tiny", fluid.CUDAPlace(0), "native", steps=2)
    assert exe._native is not None
    assert not exe._native.py_fallbacks, exe._native.py_fallbacks
    assert exe._native.host_fallbacks() == {}, exe._native.host_fallbacks()
