"""GPU probe of the grouped-expert MoE path: ernie-moe-tiny, then a mid-size config,
each stage printed as it finishes (bounded by the caller's timeout)."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from paddle_amd.models.ernie_moe import ERNIE_MOE_CONFIGS, ErnieMoEConfig, ErnieMoEForCausalLM
from paddle_amd.parallel.sharding import FlatShardedOptimizer

dev = torch.device("cuda", 0)
for name, kw, B, S in (("tiny", dict(ERNIE_MOE_CONFIGS["ernie-moe-tiny"]), 2, 64),
                       ("a3b-2l", dict(num_hidden_layers=2), 4, 2048)):
    for grouped in (False, True):
        torch.manual_seed(0)
        m = ErnieMoEForCausalLM(ErnieMoEConfig(**kw, grouped_experts=grouped), dev)
        print(name, "grouped", grouped, "built", flush=True)
        opt = FlatShardedOptimizer(m.named_parameters(), lr=1e-4)
        ids = torch.randint(0, m.cfg.vocab_size, (B, S + 1), device=dev)
        for it in range(4):
            torch.cuda.synchronize(); t = time.time()
            loss = m(ids[:, :-1], ids[:, 1:]); torch.cuda.synchronize()
            print("  fwd", it, round(loss.item(), 4), flush=True)
            loss.backward(); torch.cuda.synchronize()
            print("  bwd", it, flush=True)
            opt.step(); opt.zero_grad(); torch.cuda.synchronize()
            print("  step", it, "%.1f ms" % ((time.time() - t) * 1e3), flush=True)
        del m, opt
        torch.cuda.empty_cache()
