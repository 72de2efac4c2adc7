"""Mixture-of-Experts with expert parallelism (all-to-all token dispatch).

North-star component (SURVEY §2.5 row "Expert parallel": "No all-to-all or MoE
gating op" in the reference).  API follows Paddle's ``incubate.distributed.models
.moe.MoELayer`` (gate = "naive" / "gshard" / "switch", ``top_k``, ``l_aux``).

MI355X design:
  * routing = one [T, E] gate GEMM + softmax + top-k on device; tokens are sorted by
    destination expert with a single stable argsort (no Python loops over tokens);
  * without a capacity factor, dispatch / combine are ``all_to_all_single`` with
    exact (uneven) split sizes (one host read of the split sizes per layer);
  * with a capacity factor (GShard semantics: overflow slots dropped), tokens are
    laid out in fixed [expert, capacity] slabs and exchanged with EQUAL splits, so
    the whole layer -- routing, dispatch, exchange, grouped expert GEMMs, combine --
    runs without a single device->host sync (``sync_free=True``, the default);
  * experts on a rank run back to back on contiguous token slices; the EP group is
    meant to be the node's 8 GPUs (xGMI all-to-all is 7 concurrent P2P links).
"""
from __future__ import annotations

import torch

from ...utils import strict as _strict
import torch.nn.functional as F

from ...nn import Layer
from ...ops import moe_route as _route
from ...parallel import comm
from ...autograd import tape as _tape  # noqa: E402


class _AllToAll(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, in_splits, out_splits, group):
        ctx.in_splits, ctx.out_splits, ctx.group = in_splits, out_splits, group
        out = x.new_empty((sum(out_splits),) + tuple(x.shape[1:]))
        comm.all_to_all(out, x.contiguous(), group=group, out_splits=out_splits, in_splits=in_splits)
        return out

    @staticmethod
    def backward(ctx, g):
        out = g.new_empty((sum(ctx.in_splits),) + tuple(g.shape[1:]))
        comm.all_to_all(out, g.contiguous(), group=ctx.group, out_splits=ctx.in_splits, in_splits=ctx.out_splits)
        return out, None, None, None


def all_to_all(x, in_splits, out_splits, group):
    if comm.get_world_size(group) == 1:
        return x
    return _tape.apply(_AllToAll, x, in_splits, out_splits, group)


class _PeerExpertSwap(torch.autograd.Function):
    """[a, b, C, H] -> [b, a, C, H] row blocks (peer-major <-> expert-major)."""

    @staticmethod
    def forward(ctx, x, a, b):
        ctx.a, ctx.b = a, b
        return x.reshape(a, b, -1, x.shape[-1]).transpose(0, 1).reshape(-1, x.shape[-1]).contiguous()

    @staticmethod
    def backward(ctx, g):
        return g.reshape(ctx.b, ctx.a, -1, g.shape[-1]).transpose(0, 1).reshape(-1, g.shape[-1]).contiguous(), None, None


def _swap(x, a, b):
    return x if a == 1 or b == 1 else _tape.apply(_PeerExpertSwap, x, a, b)


class TopKGate(Layer):
    def __init__(self, d_model, num_experts, top_k=2, gate_type="gshard", capacity_factor=None, dtype="float32"):
        super().__init__("moe_gate", dtype)
        self.weight = self.create_parameter([d_model, num_experts])
        self.num_experts, self.top_k, self.gate_type = num_experts, top_k, gate_type
        self.capacity_factor = capacity_factor

    def forward(self, x):
        # framework region: the fp32 router GEMM runs on the native exact-fp32 MFMA
        # GEMM (pa_sgemm), softmax / top-k / the balance loss on the HIP kernels
        with _strict.region("moe:gate"):
            if x.is_cuda:
                # routing must be reproducible: a float-atomic split-K GEMM would let
                # near-tied experts flip between two runs of the same tokens
                from ...ops.convnd import deterministic

                with deterministic():
                    return self._route(x)
            return self._route(x)

    def _route(self, x):
        logits = x.float() @ self.weight.float()  # routing in fp32 whatever the activation dtype
        probs = F.softmax(logits, dim=-1)
        val, idx = probs.topk(self.top_k, dim=-1)
        if self.gate_type != "naive" and self.top_k > 1:
            val = val / val.sum(-1, keepdim=True).clamp_min(1e-9)
        # GShard / Switch load-balancing loss: E * sum_e(frac_tokens_e * mean_prob_e)
        me = probs.mean(0)
        ce = F.one_hot(idx[:, 0], self.num_experts).float().mean(0)
        l_aux = (me * ce).sum() * self.num_experts
        return val, idx, l_aux


class MoELayer(Layer):
    """``experts``: the LOCAL experts of this rank (``num_experts = len(experts) *
    ep_world``); global expert ``e`` lives on rank ``e // len(experts)``."""

    def __init__(self, d_model, experts, gate=None, top_k=2, group=None, capacity_factor=None,
                 gate_type="gshard", sync_free=True):
        super().__init__("moe_layer")
        self.group = group
        self.ep = comm.get_world_size(group)
        # either a list of per-expert layers (one GEMM chain each) or one grouped
        # module exposing ``forward_grouped(x_sorted, counts)`` (all local experts in
        # one batched GEMM per projection)
        self.grouped = hasattr(experts, "forward_grouped")
        self.experts = experts if self.grouped else torch.nn.ModuleList(experts)
        self.n_local = experts.num_experts if self.grouped else len(experts)
        self.num_experts = self.n_local * self.ep
        self.gate = gate or TopKGate(d_model, self.num_experts, top_k, gate_type, capacity_factor)
        self.top_k = self.gate.top_k
        self.capacity_factor = capacity_factor
        self.sync_free = sync_free
        self.l_aux = None

    def forward(self, x):
        shape = x.shape
        x = x.reshape(-1, shape[-1])
        T, k, E = x.shape[0], self.top_k, self.num_experts
        val, idx, self.l_aux = self.gate(x)
        flat_e = idx.reshape(-1)                       # [T*k] expert of each (token, slot)
        flat_w = val.reshape(-1)
        if self.capacity_factor is not None and self.sync_free:
            return self._forward_capacity(x, flat_e, flat_w, T, k, E).reshape(shape)
        keep = None
        if self.capacity_factor is not None:
            cap = max(1, int(self.capacity_factor * T * k / E))
            order = torch.argsort(flat_e, stable=True)
            se = flat_e[order]
            first = torch.searchsorted(se, se, right=False)
            rank_in_e = torch.arange(se.numel(), device=x.device) - first
            keep = torch.empty_like(flat_e, dtype=torch.bool)
            keep[order] = rank_in_e < cap
        # expert-sorted kept slots: src = token of each sorted row, pos = its inverse
        _, src, pos, e_sorted = _route.routing(flat_e, T, k, keep)
        # per global expert, from this rank (index_add: bincount would sync on its max)
        counts = torch.zeros(E, dtype=torch.int64, device=x.device).index_add_(0, e_sorted, torch.ones_like(e_sorted))
        send = _route.dispatch(x, src, pos, k)
        # exchange counts, then tokens: rank r receives, for each local expert, the
        # tokens of every peer (peer-major)
        if self.ep > 1:
            counts_all = torch.empty(self.ep * E, dtype=counts.dtype, device=counts.device)
            comm.all_gather(counts_all, counts, group=self.group)
            counts_all = counts_all.view(self.ep, E)
            r = comm.get_rank(self.group)
            lo, hi = r * self.n_local, (r + 1) * self.n_local
            in_splits = counts.view(self.ep, self.n_local).sum(1).tolist()
            recv_mat = counts_all[:, lo:hi]               # [peer, local expert]
            out_splits = recv_mat.sum(1).tolist()
            recv = all_to_all(send, in_splits, out_splits, self.group)
            # regroup peer-major -> expert-major
            per = recv_mat.reshape(-1).tolist()
            chunks = list(recv.split(per))
            by_expert = [torch.cat([chunks[p * self.n_local + e] for p in range(self.ep)])
                         for e in range(self.n_local)]
            # back to peer-major order
            sizes = [[int(recv_mat[p, e]) for p in range(self.ep)] for e in range(self.n_local)]
            if self.grouped:
                outs = list(self.experts.forward_grouped(torch.cat(by_expert),
                                                         [sum(sz) for sz in sizes]).split([sum(sz) for sz in sizes]))
            else:
                outs = [self.experts[e](by_expert[e]) if by_expert[e].shape[0] else by_expert[e]
                        for e in range(self.n_local)]
            split_out = [list(o.split(s)) for o, s in zip(outs, sizes)]
            back = torch.cat([split_out[e][p] for p in range(self.ep) for e in range(self.n_local)])
            y_sorted = all_to_all(back, out_splits, in_splits, self.group)
        elif self.grouped:
            y_sorted = self.experts.forward_grouped(send, counts)
        else:
            parts = list(send.split(counts.tolist()))
            y_sorted = torch.cat([self.experts[e](parts[e]) if parts[e].shape[0] else parts[e]
                                  for e in range(E)])
        return _route.combine(y_sorted, flat_w, pos, k).reshape(shape)

    def _forward_capacity(self, x, flat_e, flat_w, T, k, E):
        """Fixed-capacity EP layer with no host sync: send [E * cap] rows (global
        expert-major, so peer p's block is its n_local experts' slabs), equal-split
        all-to-all, experts on [n_local, ep * cap] padded rows (one grouped GEMM
        chain; padding rows are computed and never combined), equal-split return."""
        cap = max(1, int(self.capacity_factor * T * k / E))
        src, pos = _route.capacity_routing(flat_e, T, k, E, cap)
        send = _route.dispatch(x, src, pos, k)             # [E * cap, H]
        nl, ep = self.n_local, self.ep
        if ep > 1:
            splits = [nl * cap] * ep
            recv = all_to_all(send, splits, splits, self.group)  # [ep, nl, cap, H] from each peer
            xe = _swap(recv, ep, nl)                         # [nl, ep, cap, H] expert-major
        else:
            xe = send
        rows = ep * cap
        if self.grouped:
            ye = self.experts.forward_grouped(xe, [rows] * nl)
        else:
            ye = torch.cat([self.experts[e](xe[e * rows:(e + 1) * rows]) for e in range(nl)])
        if ep > 1:
            back = _swap(ye, nl, ep)                          # [ep, nl, cap, H] per destination peer
            ys = all_to_all(back, splits, splits, self.group)
        else:
            ys = ye
        return _route.combine(ys, flat_w, pos, k, padded=True)
