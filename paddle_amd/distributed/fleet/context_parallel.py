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
from ...autograd import tape as _tape  # noqa: E402


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
    qh, kh, vh = (_tape.apply(_SeqToHead, t, group) for t in (q, k, v))
    o = attn(qh, kh, vh, causal=causal, scale=scale)
    return _tape.apply(_HeadToSeq, o, group)


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
    kf, vf = _tape.apply(_GatherSeq, k, group), _tape.apply(_GatherSeq, v, group)
    if causal:
        kf, vf = kf[:, :(r + 1) * s], vf[:, :(r + 1) * s]
    return attn(q, kf, vf, causal=causal, scale=scale)


# ---------------------------------------------------------------- ring attention (zigzag)
#
# Causal context parallelism with balanced work: the sequence is cut into 2P chunks
# and rank r holds chunks r and 2P-1-r ("zigzag"), so every rank owns one early
# and one late chunk and does the same causal work (a contiguous split gives rank
# P-1 P times the work of rank 0).  K/V travel around the ring with point-to-point
# send/recv (one xGMI link per hop) issued BEFORE the current block's attention, so
# the transfer overlaps the kernel.  Per (query chunk a, key chunk b): a > b full
# attention, a == b causal, a < b skipped.  Partial outputs merge by log-sum-exp.
# Backward recomputes each block's probabilities from the GLOBAL log-sum-exp
# (flash-attention backward with the merged O / LSE), so no partial state is kept;
# dK / dV ride the ring back to their owners.


def zigzag_split(x, rank, world, dim=1):
    """Rank ``rank``'s zigzag shard of a full sequence: chunks r and 2P-1-r along dim."""
    ch = x.chunk(2 * world, dim)
    return torch.cat([ch[rank], ch[2 * world - 1 - rank]], dim)


def zigzag_merge(shards, dim=1):
    """Inverse of zigzag_split over the list of all ranks' shards."""
    P = len(shards)
    halves = [s.chunk(2, dim) for s in shards]
    order = [halves[r][0] for r in range(P)] + [halves[r][1] for r in reversed(range(P))]
    return torch.cat(order, dim)


def _attn_lse_ref(q, k, v, causal, scale):
    """Reference (torch fp32) attention returning (o, lse[B, H, Sq])."""
    Hq, Hk = q.shape[2], k.shape[2]
    if Hk != Hq:
        k = k.repeat_interleave(Hq // Hk, dim=2)
        v = v.repeat_interleave(Hq // Hk, dim=2)
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        Sq, Sk = q.shape[1], k.shape[1]
        m = torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).tril(Sk - Sq)
        s = s.masked_fill(~m, float("-inf"))
    lse = torch.logsumexp(s, -1)
    o = torch.matmul(torch.exp(s - lse.unsqueeze(-1)), vf).transpose(1, 2)
    return o.to(q.dtype), lse


def _attn_bwd_ref(q, k, v, o, do, lse, causal, scale):
    """Gradients of one (q, k/v block) pair given the GLOBAL o / lse of the rows."""
    Hq, Hk = q.shape[2], k.shape[2]
    rep = Hq // Hk
    kk = k.repeat_interleave(rep, dim=2) if rep > 1 else k
    vv = v.repeat_interleave(rep, dim=2) if rep > 1 else v
    qf, kf, vf, of, dof = (t.float().transpose(1, 2) for t in (q, kk, vv, o, do))
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        Sq, Sk = q.shape[1], k.shape[1]
        m = torch.ones(Sq, Sk, dtype=torch.bool, device=q.device).tril(Sk - Sq)
        s = s.masked_fill(~m, float("-inf"))
    p = torch.exp(s - lse.unsqueeze(-1))
    dv = torch.matmul(p.transpose(-1, -2), dof)
    dp = torch.matmul(dof, vf.transpose(-1, -2))
    delta = (dof * of).sum(-1, keepdim=True)
    ds = p * (dp - delta) * scale
    dq = torch.matmul(ds, kf)
    dk = torch.matmul(ds.transpose(-1, -2), qf)
    dq, dk, dv = (t.transpose(1, 2) for t in (dq, dk, dv))
    if rep > 1:
        B, Sk, _, D = dk.shape
        dk = dk.reshape(B, Sk, Hk, rep, D).sum(3)
        dv = dv.reshape(B, Sk, Hk, rep, D).sum(3)
    return dq, dk, dv


def _block_fwd(q, k, v, causal, scale):
    if q.is_cuda:
        from ...ops.fused import _fa_fwd

        return _fa_fwd(q, k, v, causal, scale)
    return _attn_lse_ref(q, k, v, causal, scale)


def _block_bwd(q, k, v, o, do, lse, causal, scale):
    if q.is_cuda:
        from ...ops.fused import _fa_bwd

        B, Sk, Hq, D = k.shape[0], k.shape[1], q.shape[2], q.shape[3]
        Hk = k.shape[2]
        dk = torch.empty(B, Sk, Hq, D, dtype=q.dtype, device=q.device)
        dv = torch.empty_like(dk)
        dq = _fa_bwd(q, k, v, o, do, lse, causal, scale, dk, dv)
        if Hk != Hq:
            dk = dk.view(B, Sk, Hk, Hq // Hk, D).sum(3)
            dv = dv.view(B, Sk, Hk, Hq // Hk, D).sum(3)
        return dq.float(), dk.float(), dv.float()
    dq, dk, dv = _attn_bwd_ref(q, k, v, o, do, lse, causal, scale)
    return dq.float(), dk.float(), dv.float()


def _ring_exchange(send, group):
    """Post this rank's tensor to the next rank and receive the previous rank's;
    returns (recv_tensor, [work handles])."""
    P, r = comm.get_world_size(group), comm.get_rank(group)
    nxt, prv = (r + 1) % P, (r - 1) % P
    gn = torch.distributed.get_global_rank(group, nxt) if group is not None else nxt
    gp = torch.distributed.get_global_rank(group, prv) if group is not None else prv
    recv = torch.empty_like(send)
    # framework RCCL on the comm stream (overlaps the current block's attention), or
    # batched isend/irecv on gloo
    return recv, comm.batch_p2p([("send", send, gn), ("recv", recv, gp)], group=group, async_op=True)


def _pairs(rank, src, P):
    """(local q half, kv half, causal) pairs to compute for KV from rank ``src``."""
    qc = (rank, 2 * P - 1 - rank)
    kc = (src, 2 * P - 1 - src)
    out = []
    for a in range(2):
        for b in range(2):
            if qc[a] > kc[b]:
                out.append((a, b, False))
            elif qc[a] == kc[b]:
                out.append((a, b, True))
    return out


def _merge(o_acc, lse_acc, o, lse):
    """log-sum-exp merge of a partial (o [B, s, H, D], lse [B, H, s]) into fp32 accumulators."""
    if o_acc is None:
        return o.float(), lse.float()
    new = torch.logaddexp(lse_acc, lse.float())
    w_old = torch.exp(lse_acc - new).transpose(1, 2).unsqueeze(-1)
    w_new = torch.exp(lse.float() - new).transpose(1, 2).unsqueeze(-1)
    return o_acc * w_old + o.float() * w_new, new


class _RingAttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, group, scale):
        P, r = comm.get_world_size(group), comm.get_rank(group)
        c = q.shape[1] // 2
        qh = (q[:, :c], q[:, c:])
        kv = torch.stack([k, v]).contiguous()
        acc = [[None, None], [None, None]]  # per local q half: (o, lse)
        src = r
        for step in range(P):
            nxt, works = _ring_exchange(kv, group) if step < P - 1 else (None, [])
            kh = (kv[0][:, :c], kv[0][:, c:])
            vh = (kv[1][:, :c], kv[1][:, c:])
            for a, b, causal in _pairs(r, src, P):
                o, lse = _block_fwd(qh[a], kh[b], vh[b], causal, scale)
                acc[a][0], acc[a][1] = _merge(acc[a][0], acc[a][1], o, lse)
            for w in works:
                w.wait()
            if nxt is not None:
                kv, src = nxt, (src - 1) % P
        o = torch.cat([acc[0][0], acc[1][0]], 1).to(q.dtype)
        lse = torch.cat([acc[0][1], acc[1][1]], 2).contiguous()
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.group, ctx.scale = group, scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        group, scale = ctx.group, ctx.scale
        P, r = comm.get_world_size(group), comm.get_rank(group)
        c = q.shape[1] // 2
        do = do.contiguous()
        qh, oh, doh = ((t[:, :c], t[:, c:]) for t in (q, o, do))
        qh, oh, doh = tuple(qh), tuple(oh), tuple(doh)
        lseh = (lse[:, :, :c].contiguous(), lse[:, :, c:].contiguous())
        dq = torch.zeros(q.shape, dtype=torch.float32, device=q.device)
        kv = torch.stack([k, v]).contiguous()
        dkv = torch.zeros(kv.shape, dtype=torch.float32, device=q.device)  # grads of the block we hold
        src = r
        for step in range(P):
            kh = (kv[0][:, :c], kv[0][:, c:])
            vh = (kv[1][:, :c], kv[1][:, c:])
            for a, b, causal in _pairs(r, src, P):
                gq, gk, gv = _block_bwd(qh[a], kh[b], vh[b], oh[a], doh[a], lseh[a], causal, scale)
                dq[:, a * c:(a + 1) * c] += gq
                dkv[0][:, b * c:(b + 1) * c] += gk
                dkv[1][:, b * c:(b + 1) * c] += gv
            # K/V move on; their gradient accumulator travels with them, so after P
            # hops every dK/dV is back at its owner with all contributions summed
            if P > 1:
                nkv, w1 = _ring_exchange(kv, group) if step < P - 1 else (kv, [])
                ndkv, w2 = _ring_exchange(dkv, group)
                for w in w1 + w2:
                    w.wait()
                kv, dkv, src = nkv, ndkv, (src - 1) % P
        return dq.to(q.dtype), dkv[0].to(k.dtype), dkv[1].to(v.dtype), None, None


def ring_attention(q, k, v, group, causal=True, scale=None):
    """Causal ring attention over zigzag shards: q, k, v are this rank's
    ``zigzag_split`` [B, 2c, H, D] slices (GQA: fewer k/v heads); returns the
    local output in the same layout.  Work per rank is balanced exactly."""
    if not causal:
        raise NotImplementedError("ring_attention implements the causal (zigzag) schedule")
    import math

    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    if comm.get_world_size(group) == 1:
        return (ops.flash_attention if q.is_cuda else _attn_ref_causal)(q, k, v, causal=True, scale=scale)
    if q.shape[1] % 2:
        raise ValueError("zigzag shards hold two equal chunks: local length must be even")
    return _tape.apply(_RingAttnFn, q, k, v, group, scale)


def _attn_ref_causal(q, k, v, causal=True, scale=None):
    return _attn_lse_ref(q, k, v, causal, scale)[0]
