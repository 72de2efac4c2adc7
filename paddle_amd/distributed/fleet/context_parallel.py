"""Sequence / context parallelism for attention ("sep" axis).

North-star component (SURVEY §2.5 row "Sequence parallel / context parallel /
ring attention / Ulysses": absent; the reference handles long sequences only via
LoD variable-length batching).

Two schemes over the sep process group (tokens of a sequence split contiguously,
rank r holding positions [r*s, (r+1)*s)):

* ``ulysses_attention`` (DeepSpeed-Ulysses): two all-to-alls turn the
  sequence split into a head split, full-length attention runs on H/P heads with
  the unchanged flash-attention kernel, and two all-to-alls turn it back.  Wire
  bytes per GPU ~ 4 x activations / P, independent of sequence length -- the right
  choice inside an xGMI node (all-to-all uses all 7 links at once).
* ``allgather_kv_attention`` (Llama-3-style context parallel): K/V are
  all-gathered along the sequence, rank r attends its queries to keys [0, (r+1)s)
  -- with that truncation the kernel's bottom-right causal alignment is exactly
  the global causal mask -- and dK/dV are reduce-scattered back.  Works for any
  head count (GQA with few KV heads) where Ulysses needs H % P == 0.
"""
from __future__ import annotations

import torch

from ... import ops
from ...parallel import comm


def _a2a(x, group):
    out = torch.empty_like(x)
    comm.all_to_all(out, x.contiguous(), group=group)
    return out


class _SeqToHead(torch.autograd.Function):
    """[B, s, H, D] (seq-split) -> [B, P*s, H/P, D] (head-split)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        P = comm.get_world_size(group)
        B, s, H, D = x.shape
        t = x.reshape(B, s, P, H // P, D).permute(2, 0, 1, 3, 4).contiguous()   # [P, B, s, H/P, D]
        t = _a2a(t.view(P, -1), group).view(P, B, s, H // P, D)               # chunk p = seq block p
        return t.permute(1, 0, 2, 3, 4).reshape(B, P * s, H // P, D)

    @staticmethod
    def backward(ctx, g):
        return _HeadToSeq.forward(ctx, g, ctx.group), None


class _HeadToSeq(torch.autograd.Function):
    """[B, P*s, H/P, D] -> [B, s, H, D]."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        P = comm.get_world_size(group)
        B, S, h, D = x.shape
        s = S // P
        t = x.reshape(B, P, s, h, D).permute(1, 0, 2, 3, 4).contiguous()        # [P(seq blk), B, s, h, D]
        t = _a2a(t.view(P, -1), group).view(P, B, s, h, D)                     # chunk p = head block p
        return t.permute(1, 2, 0, 3, 4).reshape(B, s, P * h, D)

    @staticmethod
    def backward(ctx, g):
        return _SeqToHead.forward(ctx, g, ctx.group), None


def ulysses_attention(q, k, v, group, causal=True, scale=None, attn_fn=None):
    """q, k, v: local [B, s, H, D] slices; returns local [B, s, H, D]."""
    P = comm.get_world_size(group)
    attn = attn_fn or ops.flash_attention
    if P == 1:
        return attn(q, k, v, causal=causal, scale=scale)
    if q.shape[2] % P or k.shape[2] % P:
        raise ValueError(f"Ulysses needs heads divisible by sep degree {P}")
    qh, kh, vh = (_SeqToHead.apply(t, group) for t in (q, k, v))
    o = attn(qh, kh, vh, causal=causal, scale=scale)
    return _HeadToSeq.apply(o, group)


class _GatherSeq(torch.autograd.Function):
    """[B, s, H, D] -> [B, P*s, H, D] (all-gather), backward reduce-scatter."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        P = comm.get_world_size(group)
        B, s, H, D = x.shape
        buf = torch.empty((P, B, s, H, D), dtype=x.dtype, device=x.device)
        comm.all_gather(buf, x.contiguous(), group=group)
        return buf.permute(1, 0, 2, 3, 4).reshape(B, P * s, H, D)

    @staticmethod
    def backward(ctx, g):
        P = comm.get_world_size(ctx.group)
        B, S, H, D = g.shape
        s = S // P
        t = g.reshape(B, P, s, H, D).permute(1, 0, 2, 3, 4).contiguous()
        out = torch.empty((B, s, H, D), dtype=g.dtype, device=g.device)
        comm.reduce_scatter(out, t, group=ctx.group)
        return out, None


def allgather_kv_attention(q, k, v, group, causal=True, scale=None, attn_fn=None):
    P = comm.get_world_size(group)
    attn = attn_fn or ops.flash_attention
    if P == 1:
        return attn(q, k, v, causal=causal, scale=scale)
    r = comm.get_rank(group)
    s = q.shape[1]
    kf, vf = _GatherSeq.apply(k, group), _GatherSeq.apply(v, group)
    if causal:
        kf, vf = kf[:, :(r + 1) * s], vf[:, :(r + 1) * s]
    return attn(q, kf, vf, causal=causal, scale=scale)
