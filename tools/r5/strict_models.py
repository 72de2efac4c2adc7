"""ATen census of whole model training steps (framework tape + sharded AdamW) with every
op of the step inside one strict region: which ATen device kernels are left."""
import json
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
os.environ.setdefault("FLAGS_count_aten", "1")
os.environ.setdefault("FLAGS_strict_trace", "1")
import torch  # noqa: E402

from paddle_amd.autograd import tape  # noqa: E402
from paddle_amd.parallel.sharding import FlatShardedOptimizer  # noqa: E402
from paddle_amd.utils import strict  # noqa: E402


def build(name):
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


out = {}
for name in sys.argv[1:] or ["llama", "gpt", "ernie"]:
    torch.manual_seed(0)
    m, V = build(name)
    opt = FlatShardedOptimizer(m.named_parameters(), lr=1e-4, grad_dtype=torch.float32)
    ids = torch.randint(0, V, (2, 1025), device="cuda")
    strict.reset()  # every step counted, the first one's lazy initialisations included
    for it in range(3):
        with strict.region(f"{name}:step"):
            with tape.recording() as t:
                loss = m(ids[:, :-1], ids[:, 1:])
            t.backward(loss)
            opt.step()
            opt.zero_grad()
    torch.cuda.synchronize()
    rep = strict.report()
    out[name] = {"aten_kernels": rep["aten_kernels"], "aten_sites": rep.get("aten_sites", {}),
                 "native_ops": sum(rep.get("native_ops", {}).values()),
                 "loss": float(loss)}
    print(name, json.dumps(out[name]), flush=True)
