"""Group-sharded data parallelism, stages 1/2/3 (``group_sharded_parallel``).

Reference parity: the only optimizer-state sharding in the reference is the
ParallelExecutor ``kReduce`` strategy (each gradient reduced to ONE owner device
that runs its optimizer op, then parameters broadcast --
framework/details/multi_devices_graph_pass.cc:247 GetAppropriateDeviceID,
:660 CreateReduceOp, :490 CreateBroadcastOp).  ZeRO-2/3 are absent.

* level ``"os"`` / ``"os_g"`` (stage 1/2): :class:`paddle_amd.parallel.sharding.
  FlatShardedOptimizer` -- flat bf16 parameter/gradient buffers, bucketed
  reduce-scatter overlapped with backward, fused AdamW on the fp32 shard,
  all-gather.  (With 288 GB of HBM per MI355X the full bf16 gradient buffer of a
  7B-13B model fits, so stage 2 keeps the flat buffer and only the reduce-scatter
  semantics differ.)
* level ``"p_g_os"`` (stage 3): :class:`ShardedStage3` below.  Parameters are
  grouped into *units* (every element of every ``ModuleList`` -- i.e. each
  transformer block -- plus a root unit for the rest).  A unit's parameters are
  views into ONE flat buffer whose storage exists only while the unit runs: a
  forward pre-hook all-gathers it from the bf16 shards, the forward post-hook
  frees the storage (``untyped_storage().resize_(0)``, keeping the views -- and
  the tensors autograd saved -- valid), an identity autograd node on the unit's
  outputs re-gathers it when backward reaches the unit, and once every gradient of
  the unit has landed they are reduce-scattered (fp32) into the rank's gradient
  shard and the storage is freed again.  Optimizer state: fp32 master + moments
  for the shard only (16 B/param / W + the bf16 shard).
"""
from __future__ import annotations

import math

import torch

from ..ops import optim as fused_optim
from ..parallel import comm
from ..parallel.sharding import FlatShardedOptimizer, _no_decay
from ..autograd import tape as _tape  # noqa: E402


class _Regather(torch.autograd.Function):
    @staticmethod
    def forward(ctx, unit, *xs):
        ctx.unit = unit
        out = tuple(x.view_as(x) for x in xs)
        return out if len(out) > 1 else out[0]

    @staticmethod
    def backward(ctx, *gs):
        ctx.unit.gather()
        return (None,) + gs


class _Unit:
    ALIGN = 64

    def __init__(self, owner, name, module, params, W, r, group, nd):
        self.owner, self.name, self.module = owner, name, module
        self.W, self.r, self.group = W, r, group
        decay = [(n, p) for n, p in params if not nd(n, p)]
        nodec = [(n, p) for n, p in params if nd(n, p)]
        self.params = [p for _, p in decay + nodec]
        offs, off = [], 0
        self.decay_end = None
        for i, p in enumerate(self.params):
            if i == len(decay):
                self.decay_end = off
            off = (off + self.ALIGN - 1) // self.ALIGN * self.ALIGN
            offs.append(off)
            off += p.numel()
        if self.decay_end is None:
            self.decay_end = off
        unit = W * self.ALIGN
        self.N = max(unit, (off + unit - 1) // unit * unit)
        self.S = self.N // W
        p0 = self.params[0]
        self.dtype, self.device = p0.dtype, p0.device
        self.flat = torch.zeros(self.N, dtype=self.dtype, device=self.device)
        with torch.no_grad():
            for p, o in zip(self.params, offs):
                self.flat[o:o + p.numel()].copy_(p.detach().reshape(-1))
                p.data = self.flat[o:o + p.numel()].view_as(p)
        self.offs = offs
        lo = r * self.S
        # W == 1: the shard IS the parameter storage (never released / re-gathered)
        self.p_shard = self.flat[lo:lo + self.S] if W == 1 else self.flat[lo:lo + self.S].clone()
        self.master = self.p_shard.float()
        self.m = torch.zeros_like(self.master)
        self.v = torch.zeros_like(self.master)
        self.g_shard = torch.zeros_like(self.master)
        self.local_decay_end = min(max(self.decay_end - lo, 0), self.S)
        # which shard elements belong to tensor-parallel (mp-sharded) parameters: their
        # squares are summed across mp ranks for the global norm, the rest counted once
        dm = torch.zeros(self.N, dtype=torch.float32, device=self.device)
        for p, o in zip(self.params, offs):
            if (getattr(p, "is_distributed", False) is True):
                dm[o:o + p.numel()] = 1.0
        self.dist_mask = dm[lo:lo + self.S].clone()
        self.has_dist = bool(self.dist_mask.any())
        self.nbytes = self.flat.untyped_storage().nbytes()
        self.gathered = True
        self.ready = set()

    def gather(self):
        if self.gathered:
            return
        self.flat.untyped_storage().resize_(self.nbytes)
        comm.all_gather(self.flat, self.p_shard, group=self.group)
        self.gathered = True

    def release(self):
        if not self.gathered or self.W == 1:
            return
        self.flat.untyped_storage().resize_(0)
        self.gathered = False

    def on_grad(self, p):
        self.ready.add(id(p))
        if len(self.ready) == len(self.params):
            self.reduce_grads()

    def reduce_grads(self):
        if not self.ready:
            return
        full = torch.zeros(self.N, dtype=torch.float32, device=self.device)
        for p, o in zip(self.params, self.offs):
            if p.grad is not None:
                full[o:o + p.numel()].copy_(p.grad.reshape(-1))
                p.grad = None
        part = torch.empty(self.S, dtype=torch.float32, device=self.device)
        comm.reduce_scatter(part, full, group=self.group)
        self.g_shard += part
        self.ready.clear()
        if self.owner.training_release:
            self.release()


class ShardedStage3:
    """ZeRO-3 / FSDP-style training engine (AdamW).  ``model`` parameters must be
    identical on every rank at construction (same seed, or broadcast first)."""

    def __init__(self, model, lr=3e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.0, group=None,
                 grad_clip=None, no_decay_fn=None, *, mp_group=None, pp_group=None, dp_group=None, exclude=(),
                 norm_skip=()):
        """Composition with hybrid parallelism (fleet.distributed_model):
        ``group`` is the sharding axis; ``dp_group`` an extra data-parallel axis whose
        gradient shards are all-reduced before the step; ``mp_group`` / ``pp_group``
        complete the global gradient norm (TP-sharded parameters summed over mp,
        stages summed over pp); ``exclude``: parameters kept whole (tied weights shared
        between pipeline stages; their gradients are synced by the caller) and updated
        here with their own fp32 AdamW state; ``norm_skip``: excluded parameters
        counted on another stage."""
        self.model, self.group = model, group
        self.mp_group, self.pp_group, self.dp_group = mp_group, pp_group, dp_group
        self.dpW = comm.get_world_size(dp_group) if dp_group is not None else 1
        self.excluded = list(exclude)
        ex_ids = {id(p) for p in self.excluded}
        self.norm_skip = {id(p) for p in norm_skip}
        self.ex_state = {}
        self.W, self.r = comm.get_world_size(group), comm.get_rank(group)
        self.lr, self.betas, self.eps, self.wd, self.grad_clip = lr, betas, eps, weight_decay, grad_clip
        self.step_count = 0
        self.training_release = True
        nd = no_decay_fn or _no_decay
        named = dict(model.named_parameters())
        owner = {}
        for mname, mod in model.named_modules():
            if isinstance(mod, torch.nn.ModuleList):
                for i, child in enumerate(mod):
                    for pn, p in child.named_parameters():
                        full = f"{mname}.{i}.{pn}" if mname else f"{i}.{pn}"
                        owner.setdefault(full, (f"{mname}.{i}", child))
        groups: dict = {}
        for n, p in named.items():
            if not p.requires_grad or id(p) in ex_ids:
                continue
            key, mod = owner.get(n, ("<root>", model))
            groups.setdefault(key, (mod, []))[1].append((n, p))
        self.units = []
        for key, (mod, params) in groups.items():
            u = _Unit(self, key, mod, params, self.W, self.r, group, nd)
            self.units.append(u)
            for p in u.params:
                p.register_post_accumulate_grad_hook(lambda p, u=u: u.on_grad(p))
                # the framework's eager engine / tape fire these at the same point
                p.__dict__.setdefault("_pa_grad_ready_hooks", []).append(lambda p, u=u: u.on_grad(p))
            self._hook(u)
        for u in self.units:
            u.release()

    def _hook(self, u):
        def pre(mod, args, kwargs=None):
            u.gather()

        def post(mod, args, out):
            if not (torch.is_grad_enabled() and mod.training):
                u.release()
                return out
            u.release()
            if isinstance(out, tuple):
                idx = [i for i, o in enumerate(out) if torch.is_tensor(o) and o.requires_grad]
                if not idx:
                    return out
                res = _tape.apply(_Regather, u, *[out[i] for i in idx])
                res = res if isinstance(res, tuple) else (res,)
                lst = list(out)
                for i, t in zip(idx, res):
                    lst[i] = t
                return tuple(lst)
            if torch.is_tensor(out) and out.requires_grad:
                return _tape.apply(_Regather, u, out)
            return out

        u.module.register_forward_pre_hook(pre)
        u.module.register_forward_hook(post)

    def parameters_gathered(self):
        for u in self.units:
            u.gather()

    @torch.no_grad()
    def step(self, lr=None):
        for u in self.units:  # units with unused parameters never completed their hook
            u.reduce_grads()
        if self.dp_group is not None and self.dpW > 1:
            for u in self.units:
                comm.all_reduce(u.g_shard, group=self.dp_group)
        self.step_count += 1
        lr = self.lr if lr is None else lr
        scale = 1.0 / (self.W * self.dpW)
        dev = self.units[0].device if self.units else self.excluded[0].device
        clip = None
        if self.grad_clip:
            # squares of the AVERAGED gradient: (scale * g_shard)^2
            sq = torch.zeros(2, dtype=torch.float32, device=dev)  # [tp-sharded, replicated]
            for u in self.units:
                g2 = u.g_shard.pow(2)
                d = (g2 * u.dist_mask).sum() if u.has_dist else torch.zeros((), device=dev)
                sq[0] += d * scale * scale
                sq[1] += (g2.sum() - d) * scale * scale
            comm.all_reduce(sq, group=self.group)
            for p in self.excluded:  # whole, already averaged and identical on the sharding ranks
                if p.grad is None or id(p) in self.norm_skip:
                    continue
                sq[0 if (getattr(p, "is_distributed", False) is True) else 1] += p.grad.float().pow(2).sum()
            if self.mp_group is not None and comm.get_world_size(self.mp_group) > 1:
                comm.all_reduce(sq[:1], group=self.mp_group)
            tot = sq.sum().reshape(1)
            if self.pp_group is not None and comm.get_world_size(self.pp_group) > 1:
                comm.all_reduce(tot, group=self.pp_group)
            clip = torch.clamp(self.grad_clip / (tot.sqrt() + 1e-6), max=1.0)
        for u in self.units:
            g = u.g_shard
            if clip is not None:
                g.mul_(clip * scale)
                gs = 1.0
            else:
                gs = scale
            fused_optim.adamw_flat(u.master, g, u.m, u.v, lr=lr, beta1=self.betas[0], beta2=self.betas[1],
                                   eps=self.eps, weight_decay=self.wd, step=self.step_count,
                                   param_out=u.p_shard, decay_end=u.local_decay_end, grad_scale=gs)
            g.zero_()
        for p in self.excluded:
            if p.grad is None:
                continue
            st = self.ex_state.get(id(p))
            if st is None:
                m0 = p.detach().float().reshape(-1).clone()
                st = self.ex_state[id(p)] = (m0, torch.zeros_like(m0), torch.zeros_like(m0))
            master, m, v = st
            g = p.grad.float().reshape(-1)
            if clip is not None:
                g = g * clip
            out = p.data.view(-1) if p.is_contiguous() else None
            fused_optim.adamw_flat(master, g, m, v, lr=lr, beta1=self.betas[0], beta2=self.betas[1], eps=self.eps,
                                   weight_decay=0.0 if _no_decay("", p) else self.wd, step=self.step_count,
                                   param_out=out)
            if out is None:
                p.data.copy_(master.view_as(p))

    def zero_grad(self):
        for u in self.units:
            u.g_shard.zero_()
            for p in u.params:
                p.grad = None
        for p in self.excluded:
            p.grad = None

    clear_grad = zero_grad

    def full_state_dict(self):
        """Gathered parameters (every rank), e.g. for checkpointing."""
        self.parameters_gathered()
        sd = {k: v.detach().clone() for k, v in self.model.state_dict().items()}
        for u in self.units:
            u.release()
        return sd


def group_sharded_parallel(model, optimizer=None, level="os_g", group=None, lr=3e-4, betas=(0.9, 0.95),
                           eps=1e-8, weight_decay=0.0, grad_clip=None, bucket_mb=256):
    """Paddle-style entry point: returns ``(model, optimizer)``.  ``optimizer`` may be
    ``None`` (hyper-parameters given here) -- the engine owns the AdamW state."""
    if level in ("os", "os_g"):
        opt = FlatShardedOptimizer(model.named_parameters(), lr=lr, betas=betas, eps=eps,
                                   weight_decay=weight_decay, group=group, grad_clip=grad_clip,
                                   bucket_mb=bucket_mb, stage=1 if level == "os" else 2)
        return model, opt
    if level == "p_g_os":
        return model, ShardedStage3(model, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, group=group,
                                    grad_clip=grad_clip)
    raise ValueError(f"unknown sharding level {level!r}")
