"""GPT / ERNIE-MoE / fp8 on the HIP device: bf16 kernels and the native fp8 GEMM,
trained with the framework's optimizers and checked against an fp32 CPU oracle
of the same model, same init, same optimizer."""
import pytest
import torch

import paddle_amd
from paddle_amd.models.ernie_moe import ERNIE_MOE_CONFIGS, ErnieMoEConfig, ErnieMoEForCausalLM
from paddle_amd.models.gpt import GPT_CONFIGS, GPTConfig, GPTForCausalLM
from paddle_amd.ops import fp8

pytestmark = pytest.mark.gpu


def test_fp8_linear_runs_native_gemm_and_is_accurate(monkeypatch):
    calls = []
    orig = fp8.gemm_f8
    monkeypatch.setattr(fp8, "gemm_f8", lambda *a, **k: calls.append(a[4:7]) or orig(*a, **k))
    torch.manual_seed(0)
    x = torch.randn(256, 512, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = torch.nn.Parameter((torch.randn(512, 384, device="cuda") * 0.05).to(torch.bfloat16))
    y = fp8.fp8_linear(x, w)
    ref = x.detach().float() @ w.detach().float()
    assert ((y.float() - ref).norm() / ref.norm()).item() < 0.06
    # device path == CPU emulation of the same per-row / per-column quantisation
    ycpu = fp8.fp8_linear(x.detach().cpu().float(), w.detach().cpu().float())
    assert ((y.detach().float().cpu() - ycpu).norm() / ycpu.norm()).item() < 0.02
    g = torch.randn(256, 384, device="cuda", dtype=torch.bfloat16)
    y.backward(g)
    dx_ref = g.float() @ w.detach().float().t()
    dw_ref = x.detach().float().t() @ g.float()
    assert ((x.grad.float() - dx_ref).norm() / dx_ref.norm()).item() < 0.06   # fp8 dgrad
    assert ((w.grad.float() - dw_ref).norm() / dw_ref.norm()).item() < 0.01   # bf16 wgrad
    assert calls == [(256, 384, 512), (256, 512, 384)], calls  # forward + dgrad on pa_gemm_f8


def _train(model, ids, steps, lr=1e-3):
    opt = paddle_amd.optimizer.AdamW(learning_rate=lr, parameters=model.parameters(), weight_decay=0.0)
    losses = []
    for _ in range(steps):
        loss = model(ids[:, :-1], ids[:, 1:])
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(loss.item())
    return losses


def _oracle_vs_device(make, steps=6, tol=0.03):
    """bf16 model on the device vs the fp32 model on the CPU from the same init and
    the same framework AdamW: per-step losses agree to bf16 accuracy."""
    torch.manual_seed(0)
    ref = make("float32", "cpu")
    dev = make("bfloat16", "cuda")
    dev.load_state_dict({k: v.to(device="cuda", dtype=dev.state_dict()[k].dtype) for k, v in ref.state_dict().items()})
    ids = torch.randint(0, ref.cfg.vocab_size if hasattr(ref, "cfg") else 1000, (2, 65))
    l_ref = _train(ref, ids, steps)
    l_dev = _train(dev, ids.cuda(), steps)
    # the oracle is the fp32 CPU trajectory itself (every step, not a loss trend)
    for a, b in zip(l_ref, l_dev):
        assert abs(a - b) / abs(a) < tol, (l_ref, l_dev)
    return l_ref, l_dev


def test_gpt_bf16_train_matches_fp32_oracle():
    base = dict(GPT_CONFIGS["gpt-tiny"], hidden_size=256, num_attention_heads=2)
    _oracle_vs_device(lambda dt, d: GPTForCausalLM(GPTConfig(**base, dtype=dt), d))


def test_ernie_moe_fp8_experts_train_matches_fp32_oracle():
    c = dict(ERNIE_MOE_CONFIGS["ernie-moe-tiny"])
    c.update(hidden_size=256, num_attention_heads=2, num_key_value_heads=2, moe_intermediate_size=128,
             intermediate_size=512)
    # fp8 experts on the device vs bf16-free fp32 experts on the CPU: fp8 rounding widens the band
    _oracle_vs_device(lambda dt, d: ErnieMoEForCausalLM(ErnieMoEConfig(**c, use_fp8_experts=(d == "cuda"), dtype=dt),
                                                         d), tol=0.06)


def test_llama_fp32_on_gpu_matches_cpu():
    """fp32 LLaMA on the device (kernels are bf16: fp32 takes the plain rotary +
    attention path) against the same model on the CPU."""
    from paddle_amd.models.llama import LLAMA_CONFIGS, LlamaConfig, LlamaForCausalLM

    torch.manual_seed(0)
    cfg = LlamaConfig(**LLAMA_CONFIGS["llama-tiny"], dtype="float32")
    cpu = LlamaForCausalLM(cfg, device="cpu")
    gpu = LlamaForCausalLM(cfg, device="cuda")
    gpu.load_state_dict({k: v.cuda() for k, v in cpu.state_dict().items()})
    ids = torch.randint(0, cfg.vocab_size, (2, 33))
    lc = cpu(ids[:, :-1], ids[:, 1:])
    lg = gpu(ids[:, :-1].cuda(), ids[:, 1:].cuda())
    lc.backward()
    lg.backward()
    assert torch.isfinite(lg) and abs(lc.item() - lg.item()) < 1e-3, (lc.item(), lg.item())
    for (n, pc), pg in zip(cpu.named_parameters(), gpu.parameters()):
        rel = ((pg.grad.cpu() - pc.grad).norm() / (pc.grad.norm() + 1e-12)).item()
        assert rel < 1e-2, (n, rel)
