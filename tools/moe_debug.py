import sys; sys.path.insert(0, '/root/repo')
import torch
from paddle_amd.models.ernie_moe import ErnieMoEConfig, ERNIE_MOE_CONFIGS, ErnieMoEForCausalLM
from paddle_amd.models.llama import LlamaConfig, LLAMA_CONFIGS, LlamaForCausalLM
from paddle_amd.parallel.sharding import FlatShardedOptimizer
torch.manual_seed(0)
for name in ("ernie", "ernie_noaux", "llama"):
    if name.startswith("ernie"):
        cfg = ErnieMoEConfig(**dict(ERNIE_MOE_CONFIGS['ernie-moe-a3b-8l'], num_hidden_layers=2,
                                    aux_loss_coeff=0.0 if name == "ernie_noaux" else 1e-2))
        m = ErnieMoEForCausalLM(cfg, 'cuda')
    else:
        cfg = LlamaConfig(**dict(LLAMA_CONFIGS['llama-7b'], num_hidden_layers=2, vocab_size=103424))
        m = LlamaForCausalLM(cfg, 'cuda')
    opt = FlatShardedOptimizer(m.named_parameters(), lr=1e-4, weight_decay=0.1, grad_clip=1.0, bucket_mb=512)
    ids = torch.randint(0, cfg.vocab_size, (4, 2049), device='cuda')
    out = []
    for s in range(8):
        loss = m(ids[:, :-1], ids[:, 1:]); loss.backward(); opt.step(); opt.zero_grad(); out.append(round(loss.item(), 3))
    with torch.no_grad():
        lg = m(ids[:, :-1]).float()
        print(name, out, "logit absmax", lg.abs().max().item(), "std", lg.std().item(),
              "acc", (lg.argmax(-1) == ids[:, 1:]).float().mean().item())
    del m, opt; torch.cuda.empty_cache()
