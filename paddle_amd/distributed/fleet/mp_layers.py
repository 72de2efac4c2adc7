"""Tensor (model) parallelism: Megatron-style column/row-parallel layers.

North-star component (SURVEY §2.5 row "Tensor parallel": absent from the
reference -- ``grep column_parallel`` finds nothing).  API mirrors Fleet's
``fleet.meta_parallel`` layers: ``ColumnParallelLinear``, ``RowParallelLinear``,
``VocabParallelEmbedding``, ``ParallelCrossEntropy``.

MI355X design: one all-reduce per column->row pair (two per transformer block),
issued on the current HIP stream over RCCL/xGMI; with sequence parallelism the
all-reduce becomes reduce-scatter + all-gather on the token axis (same bytes,
1/mp of the activation memory between the pair).  TP degree is meant to stay
within one node (<= 8), where all GPU pairs have a direct xGMI link.  Weights keep
Paddle's ``[in, out]`` layout; the local GEMMs go through ``ops.linear``.
"""
from __future__ import annotations

import torch

from ... import ops
from ...nn import Layer
from ...nn import initializer as I
from ...parallel import comm
from ...autograd import tape as _tape  # noqa: E402


# ------------------------------------------------------------------ autograd comm
class _CopyToRegion(torch.autograd.Function):
    """identity forward, all-reduce of the gradient backward (``c_identity``)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous().clone()
        comm.all_reduce(g, group=ctx.group)
        return g, None


class _ReduceFromRegion(torch.autograd.Function):
    """all-reduce forward (in place on a fresh GEMM output), identity backward."""

    @staticmethod
    def forward(ctx, x, group):
        x = x.contiguous()
        comm.all_reduce(x, group=group)
        return x

    @staticmethod
    def backward(ctx, g):
        return g, None


class _GatherLastDim(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        W = comm.get_world_size(group)
        if W == 1:
            return x
        ctx.n = x.shape[-1]
        buf = torch.empty((W,) + tuple(x.shape), dtype=x.dtype, device=x.device)
        comm.all_gather(buf, x.contiguous(), group=group)
        return torch.cat(list(buf.unbind(0)), dim=-1)

    @staticmethod
    def backward(ctx, g):
        W = comm.get_world_size(ctx.group)
        if W == 1:
            return g, None
        r = comm.get_rank(ctx.group)
        return g[..., r * ctx.n:(r + 1) * ctx.n].contiguous(), None


class _AllGatherTokens(torch.autograd.Function):
    """sequence parallel: [T/mp, H] -> [T, H] forward, reduce-scatter backward."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        W = comm.get_world_size(group)
        if W == 1:
            return x
        out = torch.empty((W * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        comm.all_gather(out, x.contiguous(), group=group)
        return out

    @staticmethod
    def backward(ctx, g):
        W = comm.get_world_size(ctx.group)
        if W == 1:
            return g, None
        out = torch.empty((g.shape[0] // W,) + tuple(g.shape[1:]), dtype=g.dtype, device=g.device)
        comm.reduce_scatter(out, g.contiguous(), group=ctx.group)
        return out, None


class _ReduceScatterTokens(torch.autograd.Function):
    """sequence parallel: partial [T, H] -> summed [T/mp, H]; all-gather backward."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        W = comm.get_world_size(group)
        if W == 1:
            return x
        out = torch.empty((x.shape[0] // W,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        comm.reduce_scatter(out, x.contiguous(), group=group)
        return out

    @staticmethod
    def backward(ctx, g):
        return _AllGatherTokens.forward(ctx, g, ctx.group), None


def copy_to_region(x, group):
    return _tape.apply(_CopyToRegion, x, group) if comm.get_world_size(group) > 1 else x


def reduce_from_region(x, group):
    return _tape.apply(_ReduceFromRegion, x, group) if comm.get_world_size(group) > 1 else x


def gather_last_dim(x, group):
    return _tape.apply(_GatherLastDim, x, group)


def all_gather_tokens(x, group):
    return _tape.apply(_AllGatherTokens, x, group)


def reduce_scatter_tokens(x, group):
    return _tape.apply(_ReduceScatterTokens, x, group)


class TPGroup:
    """Handle passed to models: the mp process group plus region helpers."""

    def __init__(self, group=None, sequence_parallel=False):
        self.group = group
        self.world_size = comm.get_world_size(group)
        self.rank = comm.get_rank(group)
        self.sequence_parallel = sequence_parallel

    def copy_to_region(self, x):
        return copy_to_region(x, self.group)

    def reduce_from_region(self, x):
        return reduce_from_region(x, self.group)


# ------------------------------------------------------------------------- layers
def _mp(group):
    return comm.get_world_size(group), comm.get_rank(group)


class ColumnParallelLinear(Layer):
    """``y = x W[:, shard]`` (+ bias shard); ``gather_output`` all-gathers the columns."""

    def __init__(self, in_features, out_features, has_bias=True, gather_output=False, group=None,
                 weight_attr=None, dtype="float32"):
        super().__init__("column_parallel_linear", dtype)
        W, _ = _mp(group)
        if out_features % W:
            raise ValueError(f"out_features {out_features} not divisible by mp degree {W}")
        self.group, self.gather_output = group, gather_output
        self.out_per = out_features // W
        self.weight = self.create_parameter([in_features, self.out_per], attr=weight_attr,
                                            default_initializer=I.XavierUniform())
        self.weight.is_distributed = True
        self.bias = self.create_parameter([self.out_per], is_bias=True) if has_bias else None
        if self.bias is not None:
            self.bias.is_distributed = True

    def forward(self, x):
        x = copy_to_region(x, self.group)
        y = ops.linear(x, self.weight, self.bias)
        return gather_last_dim(y, self.group) if self.gather_output else y


class RowParallelLinear(Layer):
    """``y = allreduce(x[:, shard] W[shard, :]) + b``."""

    def __init__(self, in_features, out_features, has_bias=True, input_is_parallel=True, group=None,
                 weight_attr=None, dtype="float32"):
        super().__init__("row_parallel_linear", dtype)
        W, r = _mp(group)
        if in_features % W:
            raise ValueError(f"in_features {in_features} not divisible by mp degree {W}")
        self.group, self.input_is_parallel = group, input_is_parallel
        self.in_per = in_features // W
        self.weight = self.create_parameter([self.in_per, out_features], attr=weight_attr,
                                            default_initializer=I.XavierUniform())
        self.weight.is_distributed = True
        self.bias = self.create_parameter([out_features], is_bias=True) if has_bias else None

    def forward(self, x):
        if not self.input_is_parallel:
            W, r = _mp(self.group)
            x = x[..., r * self.in_per:(r + 1) * self.in_per]
        y = reduce_from_region(ops.linear(x, self.weight), self.group)
        return y + self.bias if self.bias is not None else y


class _VocabParallelEmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, weight, start, group):
        n = weight.shape[0]
        local = ids - start
        mask = (local < 0) | (local >= n)
        local = local.masked_fill(mask, 0)
        out = ops.embedding(local, weight.detach()) if weight.is_cuda else torch.nn.functional.embedding(local, weight)
        out = out.masked_fill(mask.unsqueeze(-1), 0).contiguous()
        comm.all_reduce(out, group=group)
        ctx.save_for_backward(local, mask)
        ctx.shape = weight.shape
        return out

    @staticmethod
    def backward(ctx, g):
        local, mask = ctx.saved_tensors
        g = g.masked_fill(mask.unsqueeze(-1), 0)
        gw = torch.zeros(ctx.shape, dtype=torch.float32, device=g.device)
        gw.index_add_(0, local.reshape(-1), g.reshape(-1, g.shape[-1]).float())
        return None, gw.to(g.dtype), None, None


def vocab_parallel_embedding(ids, weight, group):
    W, r = _mp(group)
    if W == 1:
        return ops.embedding(ids, weight)
    return _tape.apply(_VocabParallelEmbeddingFn, ids, weight, r * weight.shape[0], group)


class VocabParallelEmbedding(Layer):
    def __init__(self, num_embeddings, embedding_dim, group=None, weight_attr=None, dtype="float32"):
        super().__init__("vocab_parallel_embedding", dtype)
        W, r = _mp(group)
        if num_embeddings % W:
            raise ValueError("vocab size must be divisible by mp degree")
        self.group = group
        self.per = num_embeddings // W
        self.vocab_start = r * self.per
        self.weight = self.create_parameter([self.per, embedding_dim], attr=weight_attr,
                                            default_initializer=I.Normal(0.0, 0.02))
        self.weight.is_distributed = True

    def forward(self, ids):
        return vocab_parallel_embedding(ids, self.weight, self.group)


class _ParallelCEFn(torch.autograd.Function):
    """Cross entropy over vocab-sharded logits [N, V/mp]: 3 small all-reduces
    (max, sum-exp, target logit) instead of gathering the logits."""

    @staticmethod
    def forward(ctx, logits, label, start, group, ignore_index):
        x = logits.float()
        n = x.shape[-1]
        mx = x.max(dim=-1, keepdim=True)[0]
        comm.all_reduce(mx, op=torch.distributed.ReduceOp.MAX, group=group)
        ex = torch.exp(x - mx)
        se = ex.sum(dim=-1, keepdim=True)
        comm.all_reduce(se, group=group)
        local = label - start
        valid = label != ignore_index
        inr = (local >= 0) & (local < n) & valid
        lc = local.clamp(0, n - 1)
        tgt = torch.where(inr, x.gather(-1, lc.unsqueeze(-1)).squeeze(-1), torch.zeros_like(x[..., 0]))
        comm.all_reduce(tgt, group=group)
        loss = (torch.log(se.squeeze(-1)) + mx.squeeze(-1) - tgt) * valid
        ctx.save_for_backward(ex, se, lc, inr, valid)
        ctx.dtype = logits.dtype
        return loss

    @staticmethod
    def backward(ctx, g):
        ex, se, lc, inr, valid = ctx.saved_tensors
        p = ex / se
        p.scatter_add_(-1, lc.unsqueeze(-1), -inr.unsqueeze(-1).to(p.dtype))
        p *= (g * valid).unsqueeze(-1)
        return p.to(ctx.dtype), None, None, None, None


def parallel_cross_entropy(logits, label, group, ignore_index=-100, reduction="mean"):
    from ...ops import fused as _F

    W, r = _mp(group)
    N = logits.shape[-1]
    # the nodes take the logits as produced (any leading dims): a reshape here would be
    # a view the framework tape cannot see through
    if W == 1:
        loss = _F.cross_entropy_tokens(logits, label, ignore_index)
    else:
        loss = _tape.apply(_ParallelCEFn, logits, label, r * N, group, ignore_index)
    if reduction == "none":
        return loss
    if reduction == "sum":
        return loss.sum()
    return _F.mean_valid(loss, label, ignore_index)


class ParallelCrossEntropy(Layer):
    def __init__(self, group=None, ignore_index=-100):
        super().__init__("parallel_cross_entropy")
        self.group, self.ignore_index = group, ignore_index

    def forward(self, logits, label):
        return parallel_cross_entropy(logits, label, self.group, self.ignore_index, reduction="none")
