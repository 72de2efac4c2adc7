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


class _TopKGateFn(torch.autograd.Function):
    """Router: fp32 logits = x W, probs = softmax, top-k (renormalised for gshard /
    switch), GShard balance loss E * sum_e mean_t(probs[:, e]) * frac_e (frac_e = the
    share of tokens whose first choice is e, a constant).  Outputs (val [T, k] fp32,
    idx [T, k] int64, l_aux scalar); the backward is analytic (top-k renormalisation,
    balance term, softmax, then dX = dlogits W^T, dW = X^T dlogits), so the router
    trains on the framework tape as well as under torch autograd."""

    @staticmethod
    def forward(ctx, x, w, k, renorm):
        logits = x.float() @ w.float()
        probs = torch.softmax(logits, dim=-1)
        val, idx = probs.topk(k, dim=-1)
        s = val.sum(-1, keepdim=True).clamp_min(1e-9) if renorm else None
        valn = val / s if renorm else val
        E = w.shape[1]
        if x.is_cuda and E <= 1024:
            from ...ops import _native as N

            idx = idx.contiguous()
            frac = torch.empty(E, dtype=torch.float32, device=x.device)
            N.call("pa_moe_frac", N.ptr(idx), idx.shape[0], k, E, N.ptr(frac), N.stream())
        else:
            frac = torch.nn.functional.one_hot(idx[:, 0], E).float().mean(0)
        l_aux = (probs.mean(0) * frac).sum() * E
        ctx.save_for_backward(x, w, probs, idx, valn, s if s is not None else probs.new_ones(1), frac)
        ctx.renorm = renorm
        return valn, idx, l_aux

    @staticmethod
    def backward(ctx, dval, _didx, daux):
        x, w, probs, idx, valn, s, frac = ctx.saved_tensors
        T, E = probs.shape
        if probs.is_cuda and idx.shape[1] <= 64:
            return _TopKGateFn._backward_native(ctx, x, w, probs, idx, valn, s, frac, dval, daux)
        dprobs = torch.zeros_like(probs)
        if dval is not None:
            dval = dval.float()
            if ctx.renorm:  # v_j / sum(v): d v_j = (dval_j - sum_i dval_i valn_i) / s
                dv = (dval - (dval * valn).sum(-1, keepdim=True)) / s
            else:
                dv = dval
            dprobs.scatter_add_(1, idx, dv)
        if daux is not None:
            dprobs += daux.float() * E * frac.unsqueeze(0) / T
        dlogits = probs * (dprobs - (dprobs * probs).sum(-1, keepdim=True))
        dx = (dlogits @ w.float().t()).to(x.dtype)
        dw = (x.float().t() @ dlogits).to(w.dtype)
        return dx, dw, None, None

    @staticmethod
    def _backward_native(ctx, x, w, probs, idx, valn, s, frac, dval, daux):
        """GPU backward: ``pa_moe_gate_bwd`` fuses the top-k renormalisation, the
        scatter into dprobs, the balance term and the softmax backward into dlogits;
        the two router GEMMs and the casts run on the framework kernels (native
        region: aten_native's exact-fp32 GEMM, deterministic split-K)."""
        from ...ops import _native as N
        from ...ops.convnd import deterministic

        T, E = probs.shape
        dl = torch.empty(T, E, dtype=torch.float32, device=probs.device)
        dv = None if dval is None else dval.float().contiguous()
        da = None if daux is None else daux.float().reshape(1).contiguous()
        N.call("pa_moe_gate_bwd", N.ptr(probs), N.ptr(idx), N.ptr(valn), N.ptr(s), N.ptr(frac),
               N.ptr(dv) if dv is not None else None, N.ptr(da) if da is not None else None, T, E, idx.shape[1],
               int(ctx.renorm), N.ptr(dl), N.stream())
        with _strict.region("moe:gate:bwd"), deterministic():
            wf = w if w.dtype == torch.float32 else w.float()
            xf = x if x.dtype == torch.float32 else x.float()
            dx = dl @ wf.t()
            dw = xf.t() @ dl
            return dx.to(x.dtype), dw.to(w.dtype), None, None


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
        # routing in fp32 whatever the activation dtype; GShard / Switch balance loss
        return _tape.apply(_TopKGateFn, x, self.weight, self.top_k,
                           self.gate_type != "naive" and self.top_k > 1)


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
        from ...ops import fused as _F

        shape = x.shape
        x = _F.reshape(x, (-1, shape[-1]))
        T, k, E = x.shape[0], self.top_k, self.num_experts
        val, idx, self.l_aux = self.gate(x)
        flat_e = idx.reshape(-1)                       # [T*k] expert of each (token, slot)
        flat_w = val                                   # [T, k] gate weights (combine reads them flat)
        if self.capacity_factor is not None and self.sync_free:
            return _F.reshape(self._forward_capacity(x, flat_e, flat_w, T, k, E), shape)
        cap = None if self.capacity_factor is None else max(1, int(self.capacity_factor * T * k / E))
        # expert-sorted kept slots: src = token of each sorted row, pos = its inverse;
        # counts per global expert, from this rank
        src, pos, e_sorted, counts = _route.route(flat_e, T, k, E, cap)
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
            # regroup peer-major [peer][expert] row blocks -> expert-major with ONE row
            # permutation (a recorded node: gradients flow on the framework tape too)
            nl, ep = self.n_local, self.ep
            per = recv_mat.reshape(-1).tolist()            # block (p, e) sizes, peer-major
            st = [0]
            for n_ in per:
                st.append(st[-1] + n_)
            perm = [r for e in range(nl) for p in range(ep) for r in range(st[p * nl + e], st[p * nl + e + 1])]
            perm_t = torch.tensor(perm, dtype=torch.long, device=recv.device)
            xe = _F.row_gather(recv, perm_t)
            sizes_e = [sum(int(recv_mat[p, e]) for p in range(ep)) for e in range(nl)]
            if self.grouped:
                ye = self.experts.forward_grouped(xe, sizes_e)
            else:
                outs, o = [], 0
                for e in range(nl):
                    rows = torch.arange(o, o + sizes_e[e], device=xe.device)
                    o += sizes_e[e]
                    outs.append(self.experts[e](_F.row_gather(xe, rows)) if sizes_e[e] else _F.row_gather(xe, rows))
                ye = _F.concat_rows(outs)
            inv = torch.empty_like(perm_t)
            inv[perm_t] = torch.arange(perm_t.numel(), device=perm_t.device)
            back = _F.row_gather(ye, inv)                  # expert-major -> peer-major
            y_sorted = all_to_all(back, out_splits, in_splits, self.group)
        elif self.grouped:
            y_sorted = self.experts.forward_grouped(send, counts)
        else:
            outs, o = [], 0
            for e, n_ in enumerate(counts.tolist()):
                rows = torch.arange(o, o + n_, device=send.device)
                o += n_
                part = _F.row_gather(send, rows)
                outs.append(self.experts[e](part) if n_ else part)
            y_sorted = _F.concat_rows(outs)
        return _F.reshape(_route.combine(y_sorted, flat_w, pos, k), shape)

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
            from ...ops import fused as _F

            ye = _F.concat_rows([self.experts[e](_F.row_gather(xe, torch.arange(e * rows, (e + 1) * rows,
                                                                                  device=xe.device)))
                                 for e in range(nl)])
        if ep > 1:
            back = _swap(ye, nl, ep)                          # [ep, nl, cap, H] per destination peer
            ys = all_to_all(back, splits, splits, self.group)
        else:
            ys = ye
        return _route.combine(ys, flat_w, pos, k, padded=True)
