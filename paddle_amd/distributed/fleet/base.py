"""``fleet``: collective (hybrid-parallel) training entry points.

Fleet is the north-star API named by BASELINE.json ("LLaMA-7B Fleet
hybrid-parallel").  The reference's closest equivalents are the env-driven
``fluid.Trainer`` NCCL2 / pserver auto-transpile (python/paddle/fluid/trainer.py:
295-330, reading PADDLE_TRAINER_ID / PADDLE_TRAINERS_NUM / PADDLE_PSERVER_*) and
``DistributeTranspiler`` -- both flat data parallel.

``fleet.init(is_collective=True, strategy)`` builds the process group (RCCL) and
the ``[dp, pp, sharding, sep, mp]`` topology from ``strategy.hybrid_configs``;
``distributed_model`` wraps by the active axes (PipelineParallel /
TensorParallel / DataParallel); ``distributed_optimizer`` returns a
``HybridParallelOptimizer`` that syncs data-parallel gradients (unless the model
wrapper already did), computes the global gradient norm across mp/pp/sharding
ranks for clipping (each distributed parameter counted once), and steps.
"""
from __future__ import annotations

import math

import torch

from ...parallel import comm
from ..topology import CommunicateTopology, HybridCommunicateGroup


class DistributedStrategy:
    def __init__(self):
        self.hybrid_configs = {"dp_degree": -1, "mp_degree": 1, "pp_degree": 1, "sharding_degree": 1,
                               "sep_degree": 1}
        self.pipeline_configs = {"accumulate_steps": 1, "micro_batch_size": 1}
        self.tensor_parallel_configs = {"tensor_init_seed": -1}
        self.sharding = False
        self.sharding_configs = {"stage": 1, "sharding_degree": 1, "segment_broadcast_MB": 32}
        self.recompute = False
        self.recompute_configs = {}
        self.amp = False
        self.amp_configs = {"init_loss_scaling": 32768.0, "use_pure_fp16": False}
        self.gradient_merge = False
        self.gradient_merge_configs = {"k_steps": 1, "avg": True}
        self.fuse_all_reduce_ops = True
        self.fuse_grad_size_in_MB = 64
        self.find_unused_parameters = False
        self.lamb = self.lars = self.dgc = self.localsgd = False
        self.a_sync = False
        self.a_sync_configs = {}

    def __setattr__(self, k, v):
        if k == "hybrid_configs" and "hybrid_configs" in self.__dict__:
            d = dict(self.__dict__["hybrid_configs"])
            d.update(v)
            v = d
        object.__setattr__(self, k, v)


class _Fleet:
    def __init__(self):
        self._hcg = None
        self._strategy = None
        self._is_collective = True

    def init(self, role_maker=None, is_collective=True, strategy=None):
        self._is_collective = is_collective
        self._strategy = strategy or DistributedStrategy()
        comm.init_parallel_env()
        world = comm.get_world_size()
        hc = dict(self._strategy.hybrid_configs)
        deg = {a: int(hc.get(f"{a}_degree", 1) or 1) for a in ("mp", "pp", "sharding", "sep")}
        prod = math.prod(deg.values())
        dp = int(hc.get("dp_degree", -1))
        if dp in (-1, 0):
            if world % prod:
                raise ValueError(f"world {world} not divisible by mp*pp*sharding*sep = {prod}")
            dp = world // prod
        topo = CommunicateTopology(dict(dp=dp, **deg))
        self._hcg = HybridCommunicateGroup(topo)
        self._model_syncs_dp = False
        return self

    # ---- queries
    def get_hybrid_communicate_group(self):
        return self._hcg

    def worker_index(self):
        return comm.get_rank()

    def worker_num(self):
        return comm.get_world_size()

    def is_first_worker(self):
        return comm.get_rank() == 0

    def barrier_worker(self):
        comm.barrier()

    @property
    def user_defined_strategy(self):
        return self._strategy

    # ---- wrappers
    def distributed_model(self, model):
        hcg = self._hcg
        if hcg is None:
            raise RuntimeError("call fleet.init first")
        from .pipeline import PipelineLayer, PipelineParallel

        st = self._strategy
        stage3 = (hcg.get_sharding_parallel_world_size() > 1 and bool(getattr(st, "sharding", False))
                  and int((getattr(st, "sharding_configs", None) or {}).get("stage", 1)) == 3)
        if hcg.get_pipe_parallel_world_size() > 1:
            if not isinstance(model, PipelineLayer):
                raise TypeError("pp_degree > 1 needs a PipelineLayer model")
            wrapped = PipelineParallel(model, hcg, st)
        elif hcg.get_model_parallel_world_size() > 1:
            wrapped = TensorParallel(model, hcg, st)
        elif hcg.get_data_parallel_world_size() > 1 and hcg.get_sharding_parallel_world_size() == 1:
            from ..parallel import DataParallel

            # DataParallel reduces the gradients itself (end of every backward):
            # the optimizer wrapper must not reduce them a second time
            self._model_syncs_dp = True
            return DataParallel(model, group=hcg.get_data_parallel_group(), bucket_mb=st.fuse_grad_size_in_MB)
        else:
            wrapped = model
        if isinstance(model, PipelineLayer):
            # a tied weight held by several stages enters the global grad norm once
            # (on its first stage); its gradient is summed across them by the pipeline
            for key, p in model.shared.items():
                p._pa_norm_skip = min(model.shared_stages.get(key, {hcg.get_stage_id()})) != hcg.get_stage_id()
        if stage3:
            # ZeRO-3 on the sharding axis INSIDE the pipeline stage / TP shard: every
            # block of this stage becomes a gather-on-use unit; tied weights shared
            # with another stage stay whole (their gradients are summed across the
            # stages by the pipeline) and are counted in the norm on their first stage
            from ..sharding import ShardedStage3

            shared, skip = [], []
            if isinstance(model, PipelineLayer):
                for key, p in model.shared.items():
                    shared.append(p)
                    if min(model.shared_stages.get(key, {hcg.get_stage_id()})) != hcg.get_stage_id():
                        skip.append(p)
            dp_g = hcg.get_data_parallel_group() if hcg.get_data_parallel_world_size() > 1 else None
            wrapped._sharded = ShardedStage3(
                model, group=hcg.get_sharding_parallel_group(),
                mp_group=hcg.get_model_parallel_group() if hcg.get_model_parallel_world_size() > 1 else None,
                pp_group=hcg.get_pipe_parallel_group() if hcg.get_pipe_parallel_world_size() > 1 else None,
                dp_group=dp_g, exclude=shared, norm_skip=skip)
            self._sharded = wrapped._sharded
        return wrapped

    def distributed_optimizer(self, optimizer, strategy=None):
        if strategy is not None:
            self._strategy = strategy
        opt = HybridParallelOptimizer(optimizer, self._hcg, self._strategy, sharded=getattr(self, "_sharded", None),
                                      model_syncs_dp=getattr(self, "_model_syncs_dp", False))
        return opt

    # ---- checkpoint helpers (rank-0 writes the dp replica)
    def save_persistables(self, executor=None, dirname=None, main_program=None):
        from ... import fluid

        if comm.get_rank() == 0:
            fluid.io.save_persistables(executor, dirname, main_program)


class TensorParallel(torch.nn.Module):
    """mp > 1 (optionally with dp): broadcast replicated (non-distributed) parameters
    from the mp group's first rank so every TP rank starts from identical copies; dp
    gradient sync is left to the HybridParallelOptimizer."""

    def __init__(self, layers, hcg, strategy=None):
        super().__init__()
        self._layers = layers
        self.hcg = hcg
        g = hcg.get_model_parallel_group()
        src = hcg.get_model_parallel_group_src_rank()
        with torch.no_grad():
            for p in layers.parameters():
                if not (getattr(p, "is_distributed", False) is True):
                    comm.broadcast(p.data, src=src, group=g)

    def forward(self, *a, **k):
        return self._layers(*a, **k)


class HybridParallelOptimizer:
    """Steps the user's optimizer under hybrid parallelism.

    * ZeRO-3 (``sharded`` engine from fleet.distributed_model): the engine owns the
      AdamW state of its shards; the user optimizer's lr / betas / eps / weight decay
      / global-norm clip are handed to it, and only whole (excluded, tied) parameters
      are all-reduced here over dp x sharding before the step.
    * otherwise: bucketed all-reduce of the gradients over the dp x sharding group
      (``fuse_grad_size_in_MB`` buckets in fp32), global-norm clipping over mp / pp,
      then the user optimizer."""

    def __init__(self, optimizer, hcg, strategy, sharded=None, model_syncs_dp=False):
        self._inner = optimizer
        self._skip_dp_sync = bool(model_syncs_dp)
        self.hcg = hcg
        self.strategy = strategy
        self.grad_clip = getattr(optimizer, "_grad_clip", None) or getattr(optimizer, "grad_clip", None)
        self._sharded = sharded
        # dp x sharding all-reduce overlapped with backward: buckets fired from
        # grad-ready hooks (pipelines sync their own gradients after the last
        # micro-batch, see PipelineParallel)
        self._bucket_sync = None
        W = hcg.get_dp_sharding_world_size() if hcg else 1
        if sharded is None and W > 1 and not model_syncs_dp and (hcg.get_pipe_parallel_world_size() if hcg else 1) == 1:
            from .grad_sync import GradBucketAllReduce

            mb = int(getattr(strategy, "fuse_grad_size_in_MB", 64) or 64)
            self._bucket_sync = GradBucketAllReduce(self._params(), hcg.get_dp_sharding_group(), W, mb)
        if sharded is not None:
            max_norm = getattr(self.grad_clip, "clip_norm", self.grad_clip if isinstance(
                self.grad_clip, (int, float)) else None)
            sharded.grad_clip = max_norm
            b1 = getattr(optimizer, "_beta1", None)
            b2 = getattr(optimizer, "_beta2", None)
            if b1 is not None and b2 is not None:
                sharded.betas = (float(b1), float(b2))
            if getattr(optimizer, "_epsilon", None) is not None:
                sharded.eps = float(optimizer._epsilon)
            wd = getattr(optimizer, "_weight_decay", None)
            if isinstance(wd, (int, float)):
                sharded.wd = float(wd)

    def __getattr__(self, k):
        return getattr(self._inner, k)

    def _params(self):
        if hasattr(self._inner, "param_groups"):
            return [p for g in self._inner.param_groups for p in g["params"]]
        return list(getattr(self._inner, "_parameter_list", []) or [])

    @torch.no_grad()
    def _dp_sync(self, params):
        """Bucketed fp32 all-reduce over dp x sharding (buckets of fuse_grad_size_in_MB)."""
        hcg = self.hcg
        W = hcg.get_dp_sharding_world_size() if hcg else 1
        ps = [p for p in params if p.grad is not None]
        if W <= 1 or not ps:
            return
        limit = int(getattr(self.strategy, "fuse_grad_size_in_MB", 64) or 64) * 2**20 // 4
        group = hcg.get_dp_sharding_group()
        bucket, n = [], 0
        for i, p in enumerate(ps):
            bucket.append(p)
            n += p.numel()
            if n >= limit or i == len(ps) - 1:
                flat = torch.cat([q.grad.reshape(-1).float() for q in bucket])
                comm.all_reduce(flat, group=group)
                flat /= W
                o = 0
                for q in bucket:
                    q.grad.copy_(flat[o:o + q.numel()].view_as(q.grad))
                    o += q.numel()
                bucket, n = [], 0

    @torch.no_grad()
    def global_grad_norm(self, params):
        """sqrt(sum g^2) over the WHOLE model: distributed (TP-sharded) params are summed
        across mp ranks, replicated ones counted once; then summed across pp stages."""
        hcg = self.hcg
        dev = params[0].device if params else "cpu"
        dist_sq = torch.zeros(1, dtype=torch.float32, device=dev)
        rep_sq = torch.zeros(1, dtype=torch.float32, device=dev)
        for p in params:
            if p.grad is None or getattr(p, "_pa_norm_skip", False):
                continue
            s = p.grad.float().pow(2).sum()
            if (getattr(p, "is_distributed", False) is True):
                dist_sq += s
            else:
                rep_sq += s
        if hcg is not None and hcg.get_model_parallel_world_size() > 1:
            comm.all_reduce(dist_sq, group=hcg.get_model_parallel_group())
        tot = dist_sq + rep_sq
        if hcg is not None and hcg.get_pipe_parallel_world_size() > 1:
            comm.all_reduce(tot, group=hcg.get_pipe_parallel_group())
        return tot.sqrt()

    def step(self):
        if self._sharded is not None:
            eng = self._sharded
            # whole (tied) parameters: average over every data-parallel replica
            self._dp_sync(eng.excluded)
            lr = self._inner.get_lr() if hasattr(self._inner, "get_lr") else None
            eng.step(lr=lr)
            return
        params = self._params()
        from .pipeline import PipelineParallel  # noqa: F401  (pipeline syncs dp itself)

        if not getattr(self, "_skip_dp_sync", False):
            self._sync_grads_before_unscale()
        self._grads_synced = False
        clip = self.grad_clip
        max_norm = getattr(clip, "clip_norm", clip if isinstance(clip, (int, float)) else None)
        if max_norm:
            norm = self.global_grad_norm(params)
            coef = torch.clamp(max_norm / (norm + 1e-6), max=1.0)
            for p in params:
                if p.grad is not None:
                    p.grad.mul_(coef.to(p.grad.dtype))
        # the global (mp x pp) clip above replaces the user optimizer's own, which
        # would clip again with a local norm
        inner_clip = [(a, getattr(self._inner, a)) for a in ("_grad_clip", "grad_clip")
                      if max_norm and getattr(self._inner, a, None) is not None]
        for a, _ in inner_clip:
            setattr(self._inner, a, None)
        try:
            self._inner.step()
        finally:
            for a, v in inner_clip:
                setattr(self._inner, a, v)

    def _sync_grads_before_unscale(self):
        """Average the gradients over dp x sharding once per step.  AMP's
        ``GradScaler.unscale_`` calls this BEFORE it unscales and checks for inf, so
        every rank tests the same (reduced) gradients and takes the same skip / step
        decision; ``step()`` then finds them synced."""
        if getattr(self, "_grads_synced", False) or self._sharded is not None:
            return
        if getattr(self, "_skip_dp_sync", False):
            return
        if self._bucket_sync is not None:
            self._bucket_sync.finish()
        else:
            self._dp_sync(self._params())
        self._grads_synced = True

    def clear_grad(self, set_to_zero=False):
        self._grads_synced = False
        if self._bucket_sync is not None:
            self._bucket_sync.reset()  # drop what a skipped step (AMP inf) left pending
        if self._sharded is not None:
            self._sharded.zero_grad()
            return
        if hasattr(self._inner, "clear_grad"):
            return self._inner.clear_grad()
        return self._inner.zero_grad(set_to_none=not set_to_zero)

    zero_grad = clear_grad


fleet = _Fleet()
