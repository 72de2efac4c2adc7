"""GPT / ERNIE-MoE / fp8 on the HIP device (bf16 kernels + hipBLASLt fp8 GEMM)."""
import pytest
import torch

from paddle_amd.models.ernie_moe import ERNIE_MOE_CONFIGS, ErnieMoEConfig, ErnieMoEForCausalLM
from paddle_amd.models.gpt import GPT_CONFIGS, GPTConfig, GPTForCausalLM
from paddle_amd.ops import fp8

pytestmark = pytest.mark.gpu


def test_fp8_scaled_mm_available_and_accurate():
    assert fp8._can_scaled_mm(torch.device("cuda")), "hipBLASLt fp8 GEMM unavailable on this device"
    torch.manual_seed(0)
    x = torch.randn(256, 512, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(512, 384, device="cuda") * 0.05).to(torch.bfloat16)
    y = fp8.fp8_linear(x, w)
    ref = x.float() @ w.float()
    assert ((y.float() - ref).norm() / ref.norm()).item() < 0.06
    # device path == CPU emulation of the same quantisation
    ycpu = fp8.fp8_linear(x.cpu().float(), w.cpu().float())
    assert ((y.float().cpu() - ycpu).norm() / ycpu.norm()).item() < 0.02


def test_gpt_bf16_train_step():
    torch.manual_seed(0)
    cfg = GPTConfig(**dict(GPT_CONFIGS["gpt-tiny"], hidden_size=256, num_attention_heads=2), dtype="bfloat16")
    m = GPTForCausalLM(cfg, "cuda")
    ids = torch.randint(0, cfg.vocab_size, (2, 65), device="cuda")
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3)
    losses = []
    for _ in range(5):
        loss = m(ids[:, :-1], ids[:, 1:])
        loss.backward()
        opt.step()
        opt.zero_grad()
        losses.append(loss.item())
    assert losses[-1] < losses[0]


def test_ernie_moe_fp8_experts_train_step():
    torch.manual_seed(0)
    c = dict(ERNIE_MOE_CONFIGS["ernie-moe-tiny"])
    c.update(hidden_size=256, num_attention_heads=2, num_key_value_heads=2, moe_intermediate_size=128,
             intermediate_size=512)
    cfg = ErnieMoEConfig(**c, use_fp8_experts=True, dtype="bfloat16")
    m = ErnieMoEForCausalLM(cfg, "cuda")
    ids = torch.randint(0, cfg.vocab_size, (2, 65), device="cuda")
    opt = torch.optim.AdamW(m.parameters(), lr=1e-3)
    losses = []
    for _ in range(5):
        loss = m(ids[:, :-1], ids[:, 1:])
        loss.backward()
        opt.step()
        opt.zero_grad()
        losses.append(loss.item())
    assert losses[-1] < losses[0]


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
