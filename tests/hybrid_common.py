"""Shared pieces of the hybrid-parallel GPT tests: the single-process fp32 reference
(AdamW + global-norm clip over the same global batch) and the fleet worker for
any TP x PP x sharding layout on a chosen device."""
import math

import torch

from paddle_amd.models.gpt import GPT_CONFIGS, GPTConfig, GPTPretrainingCriterion, gpt_pipeline_descs, \
    shard_gpt_state_dict

LR, CLIP, STEPS, M, LAYERS = 2e-3, 0.05, 3, 2, 4


def cfg():
    return GPTConfig(**{**GPT_CONFIGS["gpt-tiny"], "num_hidden_layers": LAYERS}, dtype="float32")


def batch(step, B=8, S=16, V=512):
    return torch.randint(0, V, (B, S + 1), generator=torch.Generator().manual_seed(100 + step))


def reference(splits, paddle_eps=False):
    """Single process, CPU fp32: mean over ``splits`` equal micro-batches per step.
    ``paddle_eps``: the framework optimizers' Adam (reference adam_op.h:84, epsilon
    added to sqrt of the uncorrected second moment); otherwise the bias-corrected
    form the ZeRO engines use."""
    from paddle_amd.distributed.fleet.pipeline import PipelineLayer

    c = cfg()
    crit = GPTPretrainingCriterion()
    model = PipelineLayer(gpt_pipeline_descs(c, "cpu"), num_stages=1, loss_fn=crit, seed=11)
    init = {k: v.detach().clone() for k, v in model.state_dict().items()}
    params = [p for p in model.parameters() if p.requires_grad]
    st = {id(p): (torch.zeros_like(p), torch.zeros_like(p)) for p in params}
    losses = []
    for s in range(STEPS):
        tot = 0.0
        for mb in batch(s).chunk(splits):
            loss = crit(model(mb[:, :-1]), mb[:, 1:]) / splits
            loss.backward()
            tot += loss.item()
        losses.append(tot)
        with torch.no_grad():
            norm = math.sqrt(sum(float(p.grad.pow(2).sum()) for p in params if p.grad is not None))
            coef = min(1.0, CLIP / (norm + 1e-6))
            b1, b2, eps = 0.9, 0.999, 1e-5
            for p in params:
                if p.grad is None:
                    continue
                g = p.grad * coef
                m, v = st[id(p)]
                m.mul_(b1).add_(g, alpha=1 - b1)
                v.mul_(b2).addcmul_(g, g, value=1 - b2)
                c1, c2 = 1 - b1 ** (s + 1), 1 - b2 ** (s + 1)
                if paddle_eps:
                    p.addcdiv_(m, v.sqrt() + eps, value=-LR * math.sqrt(c2) / c1)
                else:
                    p.addcdiv_(m / c1, (v / c2).sqrt() + eps, value=-LR)
                p.grad = None
    return losses, init, {k: v.detach().clone() for k, v in model.state_dict().items()}


def worker(rank, world, init, mp_deg, pp_deg, sh_deg, device):
    import paddle_amd
    from paddle_amd.distributed.fleet import DistributedStrategy, TPGroup, fleet
    from paddle_amd.distributed.fleet.pipeline import PipelineLayer

    if device == "cuda":
        torch.cuda.set_device(0)  # every rank on the one GPU of the box
    st = DistributedStrategy()
    st.hybrid_configs = {"dp_degree": 1, "mp_degree": mp_deg, "pp_degree": pp_deg, "sharding_degree": sh_deg}
    if sh_deg > 1:
        st.sharding = True
        st.sharding_configs = {"stage": 3}
    st.pipeline_configs = {"accumulate_steps": M}
    fleet.init(is_collective=True, strategy=st)
    hcg = fleet.get_hybrid_communicate_group()
    assert hcg.get_model_parallel_world_size() * hcg.get_pipe_parallel_world_size() * \
        hcg.get_sharding_parallel_world_size() == world
    c = cfg()
    tp = TPGroup(hcg.get_model_parallel_group())
    layer = PipelineLayer(gpt_pipeline_descs(c, device, tp), hcg=hcg, loss_fn=GPTPretrainingCriterion(tp), seed=11)
    lo = layer.bounds[hcg.get_stage_id()]
    full = {}
    for k in layer.state_dict():
        parts = k.split(".")
        full[k] = init[".".join([parts[0], str(lo + int(parts[1]))] + parts[2:])]
    mp_r, mp_w = hcg.get_model_parallel_rank(), hcg.get_model_parallel_world_size()
    layer.load_state_dict({k: v.to(device) for k, v in shard_gpt_state_dict(full, c, mp_r, mp_w).items()})
    model = fleet.distributed_model(layer)
    inner = paddle_amd.optimizer.AdamW(learning_rate=LR, parameters=list(layer.parameters()), weight_decay=0.0,
                                       epsilon=1e-5, grad_clip=paddle_amd.optimizer.clip.ClipGradByGlobalNorm(CLIP))
    opt = fleet.distributed_optimizer(inner)
    sr, sw = hcg.get_sharding_parallel_rank(), hcg.get_sharding_parallel_world_size()
    losses = []
    for s in range(STEPS):
        b = batch(s).chunk(sw)[sr].to(device)
        if hasattr(model, "train_batch"):  # pipeline schedule (1F1B over M micro-batches)
            loss = model.train_batch((b[:, :-1], b[:, 1:]), opt)
        else:  # one stage: the same M micro-batches, accumulated by hand
            crit, loss = GPTPretrainingCriterion(tp), 0.0
            for mb in b.chunk(M):
                l_mb = crit(model(mb[:, :-1]), mb[:, 1:]) / M
                l_mb.backward()
                loss = loss + l_mb.detach()
            opt.step()
            opt.clear_grad()
        t = loss.detach().reshape(1).clone()
        if sw > 1:
            torch.distributed.all_reduce(t, group=hcg.get_sharding_parallel_group())
        losses.append(float(t) / sw)
    sd = model._sharded.full_state_dict() if getattr(model, "_sharded", None) is not None else \
        {k: v.detach().cpu() for k, v in layer.state_dict().items()}
    return losses, sd, lo, mp_r, mp_w


def check(res, ref_losses, ref_final, loss_tol, atol):
    c = cfg()
    for losses, sd, lo, mp_r, mp_w in res:
        for a, b in zip(losses, ref_losses):
            assert abs(a - b) < loss_tol, (losses, ref_losses)
        full = {}
        for k in sd:
            parts = k.split(".")
            full[k] = ref_final[".".join([parts[0], str(lo + int(parts[1]))] + parts[2:])]
        want = shard_gpt_state_dict(full, c, mp_r, mp_w)
        for k, v in sd.items():
            if "position_embeddings" in k and v.shape == want[k].shape and lo > 0:
                continue  # the head stage's copy of the shared module's position table is unused
            torch.testing.assert_close(v.float().cpu(), want[k].float(), atol=atol, rtol=1e-3, msg=k)
