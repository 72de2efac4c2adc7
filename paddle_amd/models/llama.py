"""LLaMA decoder-only transformer (the BASELINE.json flagship: LLaMA-7B).

North-star model (not in the Fluid 0.14 reference).  Paddle-side
reference behaviour is PaddleNLP's ``LlamaForCausalLM`` with
``fuse_attention_qkv`` / ``fuse_attention_ffn``: pre-RMSNorm blocks, rotary
(neox "rotate-half") positions, SwiGLU MLP, untied LM head.

MI355X design:
  * one fused QKV GEMM and one fused gate|up GEMM per block on the hand-written
    gfx950 MFMA GEMM (``csrc/kernels/gemm.hip``), weights in Paddle's ``[in, out]``
    layout;
  * rotary + causal flash attention in one autograd node on the packed QKV output
    (``ops.rope_attention``: gfx950 MFMA kernels, no q/k/v copies);
  * the residual add is fused into the following RMSNorm (``residual=`` path), so
    each block reads the residual stream once per norm;
  * SwiGLU and the vocab-sized softmax-cross-entropy are single-pass kernels; the
    CE gradient is written in place over the logits.
  * parameters are created directly on the target device in the compute dtype.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch

from .. import ops
from ..autograd import tape as _tape
from ..nn import Layer


@dataclass
class LlamaConfig:
    vocab_size: int = 32000
    hidden_size: int = 4096
    intermediate_size: int = 11008
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    num_key_value_heads: int | None = None
    max_position_embeddings: int = 2048
    rms_norm_eps: float = 1e-6
    rope_theta: float = 10000.0
    initializer_range: float = 0.02
    tie_word_embeddings: bool = False
    recompute: bool = False
    dtype: str = "bfloat16"
    # tensor parallel degree/rank (column/row split of the GEMMs); 1 = off
    tensor_parallel_degree: int = 1
    extra: dict = field(default_factory=dict)

    @property
    def head_dim(self):
        return self.hidden_size // self.num_attention_heads

    @property
    def kv_heads(self):
        return self.num_key_value_heads or self.num_attention_heads

    def num_params(self):
        H, I, V, L = self.hidden_size, self.intermediate_size, self.vocab_size, self.num_hidden_layers
        kvd = self.kv_heads * self.head_dim
        per = H * (H + 2 * kvd) + H * H + 3 * H * I + 2 * H
        return V * H * (1 if self.tie_word_embeddings else 2) + L * per + H


LLAMA_CONFIGS = {
    "llama-7b": dict(hidden_size=4096, intermediate_size=11008, num_hidden_layers=32, num_attention_heads=32),
    "llama-13b": dict(hidden_size=5120, intermediate_size=13824, num_hidden_layers=40, num_attention_heads=40),
    "llama-tiny": dict(vocab_size=512, hidden_size=256, intermediate_size=688, num_hidden_layers=2,
                       num_attention_heads=2, max_position_embeddings=256),
}


def _dt(s):
    return {"bfloat16": torch.bfloat16, "float32": torch.float32, "float16": torch.float16}[s]


def _param(shape, device, dtype, std=None, value=None):
    t = torch.empty(*shape, device=device, dtype=torch.float32)
    if value is not None:
        t.fill_(value)
    else:
        t.normal_(0.0, std)
    return torch.nn.Parameter(t.to(dtype))


def mlp_interleaved(cfg, tp=None) -> bool:
    """Whether a (non tensor-parallel) LLaMA block stores gate|up interleaved."""
    tpd = tp.world_size if tp is not None else 1
    return tpd == 1 and cfg.intermediate_size % (2 * 8) == 0


class LlamaDecoderLayer(Layer):
    def __init__(self, cfg: LlamaConfig, device=None, layer_idx=0, tp=None):
        super().__init__("llama_decoder")
        H, I = cfg.hidden_size, cfg.intermediate_size
        dt = _dt(cfg.dtype)
        std = cfg.initializer_range
        self.cfg = cfg
        self.tp = tp  # optional parallel.tensor_parallel.TPGroup
        tpd = tp.world_size if tp is not None else 1
        self.nh = cfg.num_attention_heads // tpd
        self.nkv = cfg.kv_heads // tpd
        D = cfg.head_dim
        self.input_layernorm = _param([H], device, dt, value=1.0)
        self.qkv_proj = _param([H, (self.nh + 2 * self.nkv) * D], device, dt, std)
        self.o_proj = _param([self.nh * D, H], device, dt, std / math.sqrt(2 * cfg.num_hidden_layers))
        self.post_attention_layernorm = _param([H], device, dt, value=1.0)
        self.gate_up_proj = _param([H, 2 * I // tpd], device, dt, std)
        self.down_proj = _param([I // tpd, H], device, dt, std / math.sqrt(2 * cfg.num_hidden_layers))
        for n in ("input_layernorm", "post_attention_layernorm"):
            getattr(self, n).no_weight_decay = True
        # gate|up columns interleaved in 16-column blocks (ops.interleave_gate_up) so the
        # MLP runs as one fused node; tensor-parallel shards keep [gate | up].  The
        # interleaving is an in-memory layout only: state dicts always carry the
        # canonical [gate | up] matrix (_save_to_state_dict / _pa_state_in below), so
        # checkpoints load the same whatever layout the loading model uses.
        self.mlp_interleaved = mlp_interleaved(cfg, tp)

    # state-dict format version of gate_up_proj: 2 = canonical [gate | up] (always)
    _version = 2

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        super()._save_to_state_dict(destination, prefix, keep_vars)
        k = prefix + "gate_up_proj"
        if self.mlp_interleaved and k in destination:
            g, u = ops.deinterleave_gate_up(destination[k].detach())
            destination[k] = torch.cat([g, u], -1)

    def _pa_state_in(self, name, value):
        """Canonical [gate | up] checkpoint tensor -> this layer's in-memory layout."""
        if name == "gate_up_proj" and self.mlp_interleaved:
            I = value.shape[-1] // 2
            return ops.interleave_gate_up(value[..., :I], value[..., I:])
        return value

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing, unexpected, errors):
        k = prefix + "gate_up_proj"
        if k in state_dict:
            state_dict = dict(state_dict)
            state_dict[k] = self._pa_state_in("gate_up_proj", state_dict[k])
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing, unexpected, errors)

    def forward(self, x, residual, cos, sin):
        cfg = self.cfg
        eps = cfg.rms_norm_eps
        if residual is None:
            h = x
            y = ops.rms_norm(x, self.input_layernorm, eps)
        else:
            y, h = ops.rms_norm(x, self.input_layernorm, eps, residual=residual)
        if self.tp is not None:
            y = self.tp.copy_to_region(y)
        # QKV projection with the rotary in its epilogue, then flash attention (one node)
        a = ops.qkv_rope_attention(y, self.qkv_proj, cos, sin, self.nh, self.nkv, causal=True)
        a = ops.linear(a, self.o_proj)
        if self.tp is not None:
            a = self.tp.reduce_from_region(a)
        y2, h2 = ops.rms_norm(a, self.post_attention_layernorm, eps, residual=h)
        if self.tp is not None:
            y2 = self.tp.copy_to_region(y2)
        if self.mlp_interleaved:
            m = ops.swiglu_mlp(y2, self.gate_up_proj, self.down_proj)
        else:
            m = ops.linear(ops.swiglu(ops.linear(y2, self.gate_up_proj)), self.down_proj)
        if self.tp is not None:
            m = self.tp.reduce_from_region(m)
        return m, h2


class LlamaForCausalLM(Layer):
    """``tp``: optional ``distributed.fleet.TPGroup`` -- Megatron tensor parallelism:
    QKV / gate|up column-parallel, o / down row-parallel (one all-reduce each),
    vocab-parallel embedding, vocab-sharded LM head + parallel cross entropy."""

    def __init__(self, cfg: LlamaConfig, device=None, tp=None):
        super().__init__("llama")
        self.cfg = cfg
        self.tp = tp if (tp is not None and tp.world_size > 1) else None
        dt = _dt(cfg.dtype)
        std = cfg.initializer_range
        H = cfg.hidden_size
        tpd = self.tp.world_size if self.tp else 1
        if cfg.vocab_size % tpd:
            raise ValueError("vocab_size must be divisible by the tensor-parallel degree")
        self.embed_tokens = _param([cfg.vocab_size // tpd, H], device, dt, std)
        self.layers = torch.nn.ModuleList(
            [LlamaDecoderLayer(cfg, device, i, self.tp) for i in range(cfg.num_hidden_layers)])
        self.norm = _param([H], device, dt, value=1.0)
        self.norm.no_weight_decay = True
        self.lm_head = None if cfg.tie_word_embeddings else _param([H, cfg.vocab_size // tpd], device, dt, std)
        if self.tp:
            for name, prm in self.named_parameters():
                if prm.dim() == 2:
                    prm.is_distributed = True
        cos, sin = ops.rope_tables(cfg.max_position_embeddings, cfg.head_dim, cfg.rope_theta, device=device)
        self.register_buffer("rope_cos", cos, persistent=False)
        self.register_buffer("rope_sin", sin, persistent=False)

    def embed(self, input_ids):
        if self.tp:
            from ..distributed.fleet.mp_layers import vocab_parallel_embedding

            return vocab_parallel_embedding(input_ids, self.embed_tokens, self.tp.group)
        return ops.embedding(input_ids, self.embed_tokens)

    def hidden_states(self, input_ids):
        x = self.embed(input_ids)
        residual = None
        cos, sin = self.rope_cos, self.rope_sin
        for layer in self.layers:
            if self.cfg.recompute and self.training and _tape.current() is not None:
                x, residual = _tape.checkpoint(layer, x, residual, cos, sin)  # recomputed on the framework tape
            elif self.cfg.recompute and self.training and torch.is_grad_enabled():
                x, residual = torch.utils.checkpoint.checkpoint(layer, x, residual, cos, sin,
                                                                use_reentrant=False)
            else:
                x, residual = layer(x, residual, cos, sin)
        y, _ = ops.rms_norm(x, self.norm, self.cfg.rms_norm_eps, residual=residual)
        return y

    def logits_and_loss(self, y, labels):
        if self.tp:
            from ..distributed.fleet.mp_layers import parallel_cross_entropy

            logits = ops.linear(self.tp.copy_to_region(y), self.lm_head)
            if labels is None:
                return logits
            return parallel_cross_entropy(logits, labels, self.tp.group)
        if self.lm_head is not None:
            logits = ops.linear(y, self.lm_head)
        else:
            logits = ops.linear_t(y, self.embed_tokens)
        if labels is None:
            return logits
        # in-place CE gradient over the logits buffer (nothing else consumes it)
        return ops.softmax_cross_entropy(logits, labels, inplace_grad=True)

    def forward(self, input_ids, labels=None):
        return self.logits_and_loss(self.hidden_states(input_ids), labels)


def shard_llama_state_dict(full: dict, cfg: LlamaConfig, rank: int, world: int) -> dict:
    """Full (single-rank) LLaMA state dict -> tensor-parallel shard ``rank`` of ``world``
    (column splits keep the [q|k|v] and [gate|up] packing per rank).  ``full`` is in
    the canonical state-dict layout ([gate | up], ``LlamaDecoderLayer._version`` 2)."""
    if world == 1:
        return dict(full)
    D = cfg.head_dim
    nh, nkv, I = cfg.num_attention_heads, cfg.kv_heads, cfg.intermediate_size
    out = {}
    for k, v in full.items():
        if k.endswith("qkv_proj"):
            q, kk, vv = v.split([nh * D, nkv * D, nkv * D], dim=1)
            out[k] = torch.cat([t.chunk(world, dim=1)[rank] for t in (q, kk, vv)], dim=1).contiguous()
        elif k.endswith("gate_up_proj"):
            g, u = v.split([I, I], dim=1)
            out[k] = torch.cat([g.chunk(world, dim=1)[rank], u.chunk(world, dim=1)[rank]], dim=1).contiguous()
        elif k.endswith("o_proj") or k.endswith("down_proj") or k == "embed_tokens":
            out[k] = v.chunk(world, dim=0)[rank].contiguous()
        elif k == "lm_head":
            out[k] = v.chunk(world, dim=1)[rank].contiguous()
        else:
            out[k] = v.clone()
    return out


# ---------------------------------------------------------------- pipeline stages
class LlamaEmbeddingPipe(Layer):
    def __init__(self, cfg: LlamaConfig, device=None, tp=None):
        super().__init__("llama_embed_pipe")
        self.cfg = cfg
        self.tp = tp if (tp is not None and tp.world_size > 1) else None
        tpd = self.tp.world_size if self.tp else 1
        self.embed_tokens = _param([cfg.vocab_size // tpd, cfg.hidden_size], device, _dt(cfg.dtype),
                                   cfg.initializer_range)

    def forward(self, input_ids):
        if self.tp:
            from ..distributed.fleet.mp_layers import vocab_parallel_embedding

            return vocab_parallel_embedding(input_ids, self.embed_tokens, self.tp.group)
        return ops.embedding(input_ids, self.embed_tokens)


class LlamaDecoderLayerPipe(LlamaDecoderLayer):
    """Decoder block speaking the pipeline tuple protocol: (x[, residual]) -> (x, residual)."""

    def __init__(self, cfg: LlamaConfig, device=None, layer_idx=0, tp=None):
        super().__init__(cfg, device, layer_idx, tp if (tp is not None and tp.world_size > 1) else None)
        cos, sin = ops.rope_tables(cfg.max_position_embeddings, cfg.head_dim, cfg.rope_theta, device=device)
        self.register_buffer("rope_cos", cos, persistent=False)
        self.register_buffer("rope_sin", sin, persistent=False)

    def forward(self, x, residual=None):
        return super().forward(x, residual, self.rope_cos, self.rope_sin)


class LlamaNormHeadPipe(Layer):
    def __init__(self, cfg: LlamaConfig, device=None, tp=None):
        super().__init__("llama_head_pipe")
        self.cfg = cfg
        self.tp = tp if (tp is not None and tp.world_size > 1) else None
        tpd = self.tp.world_size if self.tp else 1
        dt = _dt(cfg.dtype)
        self.norm = _param([cfg.hidden_size], device, dt, value=1.0)
        self.norm.no_weight_decay = True
        self.lm_head = _param([cfg.hidden_size, cfg.vocab_size // tpd], device, dt, cfg.initializer_range)

    def forward(self, x, residual):
        y, _ = ops.rms_norm(x, self.norm, self.cfg.rms_norm_eps, residual=residual)
        if self.tp:
            y = self.tp.copy_to_region(y)
        return ops.linear(y, self.lm_head)


class LlamaPretrainingCriterion:
    def __init__(self, tp=None):
        self.tp = tp if (tp is not None and tp.world_size > 1) else None

    def __call__(self, logits, labels):
        if self.tp:
            from ..distributed.fleet.mp_layers import parallel_cross_entropy

            return parallel_cross_entropy(logits, labels, self.tp.group)
        return ops.softmax_cross_entropy(logits, labels, inplace_grad=True)


def llama_pipeline_descs(cfg: LlamaConfig, device=None, tp=None):
    from ..distributed.fleet.pipeline import LayerDesc

    descs = [LayerDesc(LlamaEmbeddingPipe, cfg, device, tp)]
    descs += [LayerDesc(LlamaDecoderLayerPipe, cfg, device, i, tp) for i in range(cfg.num_hidden_layers)]
    descs.append(LayerDesc(LlamaNormHeadPipe, cfg, device, tp))
    return descs


def llama_flops_per_token(cfg: LlamaConfig, seq_len: int) -> float:
    """Training FLOPs per token (fwd+bwd = 3x fwd), dense GEMMs + causal attention."""
    H, I, L, V = cfg.hidden_size, cfg.intermediate_size, cfg.num_hidden_layers, cfg.vocab_size
    kvd = cfg.kv_heads * cfg.head_dim
    gemm = 2 * (H * (H + 2 * kvd) + H * H + 3 * H * I)
    attn = 2 * 2 * seq_len * H / 2  # QK^T + PV, causal half
    return 3 * (L * (gemm + attn) + 2 * H * V)
