"""Process-group bootstrap and collective helpers (RCCL over xGMI on MI355X).

One process per GPU (``torch.distributed`` backend ``nccl`` == RCCL on ROCm);
``gloo`` on CPU for tests.  Replaces the reference's single-process
``NCCLContextMap`` (paddle/fluid/platform/nccl_helper.h:81-123) and the
``gen_nccl_id`` gRPC rendezvous (operators/gen_nccl_id_op.cc:54-110) with a TCP
store rendezvous driven by the standard RANK/WORLD_SIZE/MASTER_* env (also
accepting Paddle's PADDLE_TRAINER_ID / PADDLE_TRAINERS_NUM).
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist

_GROUPS: dict = {}


def env_rank_world():
    rank = int(os.environ.get("RANK", os.environ.get("PADDLE_TRAINER_ID", "0")))
    world = int(os.environ.get("WORLD_SIZE", os.environ.get("PADDLE_TRAINERS_NUM", "1")))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, world, local


def init_parallel_env(backend: str | None = None, timeout_s: float = 1800.0):
    """Initialise the default process group once (idempotent).  Returns (rank, world)."""
    rank, world, local = env_rank_world()
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    if world <= 1:
        return 0, 1
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    kw = {}
    if backend == "nccl":
        kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
    dist.init_process_group(backend, rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return rank, world


def is_dist():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


class _SelfGroup:
    """A one-rank group (an axis of degree 1 in a hybrid topology).  ``None`` means
    the WORLD group everywhere in this module, so size-1 axes need their own token."""

    def __repr__(self):
        return "SELF"


SELF = _SelfGroup()


def get_rank(group=None):
    if group is SELF:
        return 0
    return dist.get_rank(group) if is_dist() else 0


def get_world_size(group=None):
    if group is SELF:
        return 1
    return dist.get_world_size(group) if is_dist() else 1


def _is_gloo(group=None):
    return dist.get_backend(group) == "gloo"


def _pa_comm(group, *ts):
    """The framework-owned RCCL communicator of ``group`` (FLAGS_comm_backend=pa_rccl)
    when every operand is a contiguous device tensor, else None (torch.distributed)."""
    from . import rccl

    if not rccl.enabled() or not all(t.is_cuda and t.is_contiguous() for t in ts):
        return None
    ranks = list(range(dist.get_world_size())) if group is None else dist.get_process_group_ranks(group)
    return rccl.context_map().get(ranks, dist.get_rank())


def all_reduce(t, op=dist.ReduceOp.SUM, group=None, async_op=False):
    if get_world_size(group) == 1:
        return None
    c = _pa_comm(group, t) if op == dist.ReduceOp.SUM else None
    if c is not None:
        c.all_reduce(t)  # stream-ordered on the current stream: nothing to wait for
        return None
    return dist.all_reduce(t, op=op, group=group, async_op=async_op)


def reduce_scatter(out, inp, group=None, async_op=False):
    """out (numel = inp.numel()/W) = this rank's chunk of sum_r inp_r."""
    W = get_world_size(group)
    if W == 1:
        out.copy_(inp)
        return None
    if _is_gloo(group):
        tmp = inp.clone()
        dist.all_reduce(tmp, group=group)
        r = dist.get_rank(group)
        n = out.numel()
        out.copy_(tmp.view(-1)[r * n:(r + 1) * n].view_as(out))
        return None
    c = _pa_comm(group, out, inp)
    if c is not None:
        c.reduce_scatter(out, inp)
        return None
    return dist.reduce_scatter_tensor(out, inp, group=group, async_op=async_op)


def all_gather(out, inp, group=None, async_op=False):
    """out = concat_r inp_r (rank order)."""
    W = get_world_size(group)
    if W == 1:
        out.copy_(inp)
        return None
    if _is_gloo(group):
        chunks = list(out.view(W, -1).unbind(0))
        tmp = [torch.empty_like(c) for c in chunks]
        dist.all_gather(tmp, inp.contiguous().view(-1), group=group)
        for c, t in zip(chunks, tmp):
            c.copy_(t)
        return None
    c = _pa_comm(group, out, inp)
    if c is not None:
        c.all_gather(out, inp)
        return None
    return dist.all_gather_into_tensor(out, inp, group=group, async_op=async_op)


def broadcast(t, src=0, group=None):
    if get_world_size(group) == 1:
        return
    c = _pa_comm(group, t)
    if c is not None:
        ranks = list(range(dist.get_world_size())) if group is None else dist.get_process_group_ranks(group)
        c.broadcast(t, root=ranks.index(src))  # src is a global rank
        return
    dist.broadcast(t, src=src, group=group)


def all_to_all(out, inp, group=None, out_splits=None, in_splits=None):
    if get_world_size(group) == 1:
        out.copy_(inp)
        return
    if _is_gloo(group):
        W = get_world_size(group)
        ins = list(inp.split(in_splits or [inp.shape[0] // W] * W))
        outs = list(out.split(out_splits or [out.shape[0] // W] * W))
        # gloo has no all_to_all: emulate with per-peer broadcast-free send/recv
        r = dist.get_rank(group)
        reqs = []
        for p in range(W):
            if p == r:
                outs[p].copy_(ins[p])
                continue
            reqs.append(dist.isend(ins[p].contiguous(), dist.get_global_rank(group, p) if group else p, group=group))
            reqs.append(dist.irecv(outs[p], dist.get_global_rank(group, p) if group else p, group=group))
        for q in reqs:
            q.wait()
        return
    dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)


def new_group(ranks):
    key = tuple(sorted(ranks))
    if key not in _GROUPS:
        _GROUPS[key] = dist.new_group(list(key))
    return _GROUPS[key]


def barrier(group=None):
    if group is SELF:
        return
    if is_dist():
        if dist.get_backend(group) == "nccl":
            dist.barrier(group=group, device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier(group=group)
