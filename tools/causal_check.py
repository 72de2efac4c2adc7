import sys; sys.path.insert(0, '/root/repo')
import torch
from paddle_amd import ops
from paddle_amd.ops.fused import _attn_ref, _rope_ref
torch.manual_seed(0)
B,S,Hq,Hk,D = 2,256,20,4,128
qkv = torch.randn(B,S,(Hq+2*Hk)*D, device='cuda', dtype=torch.bfloat16)
cos, sin = ops.rope_tables(S, D, 500000.0, device='cuda')
o = ops.rope_attention(qkv, cos, sin, Hq, Hk, causal=True)
q,k,v = qkv.float().split([Hq*D,Hk*D,Hk*D], -1)
q = _rope_ref(q.view(B,S,Hq,D), cos, sin); k = _rope_ref(k.view(B,S,Hk,D), cos, sin)
ref = _attn_ref(q, k, v.view(B,S,Hk,D), True, D**-0.5)
print("gqa rope_attention max err", (o.float().view_as(ref)-ref).abs().max().item())
qkv2 = qkv.clone(); qkv2[:, 200:] = torch.randn_like(qkv2[:, 200:])
o2 = ops.rope_attention(qkv2, cos, sin, Hq, Hk, causal=True)
print("leak into <200 from >=200:", (o2[:, :200].float()-o[:, :200].float()).abs().max().item())
from paddle_amd.models.ernie_moe import ErnieMoEConfig, ERNIE_MOE_CONFIGS, ErnieMoEForCausalLM
cfg = ErnieMoEConfig(**dict(ERNIE_MOE_CONFIGS['ernie-moe-a3b-8l'], num_hidden_layers=2))
m = ErnieMoEForCausalLM(cfg, 'cuda')
ids = torch.randint(0, cfg.vocab_size, (2, 257), device='cuda')
with torch.no_grad():
    l1 = m(ids[:, :-1]); ids2 = ids.clone(); ids2[:, 150:] = torch.randint(0, cfg.vocab_size, (2, 107), device='cuda')
    l2 = m(ids2[:, :-1])
print("model leak:", (l1[:, :150].float()-l2[:, :150].float()).abs().max().item())
loss = m(ids[:, :-1], ids[:, 1:]); print("init loss", loss.item())
