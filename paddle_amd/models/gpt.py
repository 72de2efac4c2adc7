"""GPT-3 family (decoder-only, LayerNorm + GELU MLP, learned positions, tied
embeddings) -- BASELINE.json config "GPT-3 13B Fleet hybrid parallel TP=2 PP=2
sharding stage-3".

Not in the Fluid 0.14 reference; Paddle-side behaviour follows
PaddleNLP's ``GPTForPretraining``.  MI355X design mirrors :mod:`.llama`:
  * fused QKV ``[H, 3H]`` and MLP ``[H, 4H]`` GEMMs on the hand-written MFMA GEMM
    (``csrc/kernels/gemm.hip``), Paddle ``[in, out]`` weights; attention runs the gfx950 flash kernel directly on strided q/k/v views
    of the packed QKV output (no copies);
  * the residual add is fused into the following LayerNorm kernel;
  * Megatron TP (column QKV / fc1, row o-proj / fc2, vocab-parallel embedding and
    tied LM head with parallel cross entropy) through a ``TPGroup``;
  * ``gpt_pipeline_descs`` cuts the model for 1F1B with the tied embedding as a
    ``SharedLayerDesc`` between the first and last stage.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from .. import ops
from ..autograd import tape as _tape
from ..nn import Layer
from .llama import _dt, _param


@dataclass
class GPTConfig:
    vocab_size: int = 50304
    hidden_size: int = 5120
    num_hidden_layers: int = 40
    num_attention_heads: int = 40
    intermediate_size: int | None = None
    max_position_embeddings: int = 2048
    layer_norm_eps: float = 1e-5
    initializer_range: float = 0.02
    hidden_dropout_prob: float = 0.0
    recompute: bool = False
    dtype: str = "bfloat16"

    @property
    def ffn(self):
        return self.intermediate_size or 4 * self.hidden_size

    @property
    def head_dim(self):
        return self.hidden_size // self.num_attention_heads

    def num_params(self):
        H, L = self.hidden_size, self.num_hidden_layers
        return self.vocab_size * H + self.max_position_embeddings * H + L * (
            3 * H * H + 3 * H + H * H + H + 2 * H * self.ffn + self.ffn + H + 4 * H) + 2 * H


GPT_CONFIGS = {
    "gpt3-13b": dict(hidden_size=5120, num_hidden_layers=40, num_attention_heads=40),
    "gpt3-6.7b": dict(hidden_size=4096, num_hidden_layers=32, num_attention_heads=32),
    "gpt3-1.3b": dict(hidden_size=2048, num_hidden_layers=24, num_attention_heads=16),
    "gpt3-350m": dict(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16),
    "gpt-tiny": dict(vocab_size=512, hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                     max_position_embeddings=128),
}


def _tp_on(tp):
    return tp if (tp is not None and tp.world_size > 1) else None


class GPTDecoderLayer(Layer):
    def __init__(self, cfg: GPTConfig, device=None, layer_idx=0, tp=None):
        super().__init__("gpt_decoder")
        self.cfg, self.tp = cfg, _tp_on(tp)
        tpd = self.tp.world_size if self.tp else 1
        H, I, dt, std = cfg.hidden_size, cfg.ffn, _dt(cfg.dtype), cfg.initializer_range
        out_std = std / math.sqrt(2 * cfg.num_hidden_layers)
        self.nh = cfg.num_attention_heads // tpd
        D = cfg.head_dim
        self.ln1_w = _param([H], device, dt, value=1.0)
        self.ln1_b = _param([H], device, dt, value=0.0)
        self.qkv_w = _param([H, 3 * self.nh * D], device, dt, std)
        self.qkv_b = _param([3 * self.nh * D], device, dt, value=0.0)
        self.out_w = _param([self.nh * D, H], device, dt, out_std)
        self.out_b = _param([H], device, dt, value=0.0)
        self.ln2_w = _param([H], device, dt, value=1.0)
        self.ln2_b = _param([H], device, dt, value=0.0)
        self.fc1_w = _param([H, I // tpd], device, dt, std)
        self.fc1_b = _param([I // tpd], device, dt, value=0.0)
        self.fc2_w = _param([I // tpd, H], device, dt, out_std)
        self.fc2_b = _param([H], device, dt, value=0.0)
        for n in ("ln1_w", "ln1_b", "ln2_w", "ln2_b", "qkv_b", "out_b", "fc1_b", "fc2_b"):
            getattr(self, n).no_weight_decay = True
        if self.tp:
            for n in ("qkv_w", "qkv_b", "out_w", "fc1_w", "fc1_b", "fc2_w"):
                getattr(self, n).is_distributed = True

    def _row_linear(self, x, w, b):
        # bias of a row-parallel GEMM is added once, after the all-reduce; without
        # TP it rides the GEMM epilogue
        if not self.tp:
            return ops.linear(x, w, b)
        return ops.add(self.tp.reduce_from_region(ops.linear(x, w)), b)

    def forward(self, x, residual=None):
        cfg, eps = self.cfg, self.cfg.layer_norm_eps
        if residual is None:
            h = x
            y = ops.layer_norm(x, self.ln1_w, self.ln1_b, eps)
        else:
            y, h = ops.layer_norm(x, self.ln1_w, self.ln1_b, eps, residual=residual)
        if self.tp:
            y = self.tp.copy_to_region(y)
        # packed q|k|v straight into the attention kernel; dqkv comes back packed
        a = ops.packed_attention(ops.linear(y, self.qkv_w, self.qkv_b), self.nh, causal=True)
        a = self._row_linear(a, self.out_w, self.out_b)
        y2, h2 = ops.layer_norm(a, self.ln2_w, self.ln2_b, eps, residual=h)
        if self.tp:
            y2 = self.tp.copy_to_region(y2)
        m = self._row_linear(ops.linear_gelu(y2, self.fc1_w, self.fc1_b), self.fc2_w, self.fc2_b)
        return m, h2


class GPTEmbeddings(Layer):
    def __init__(self, cfg: GPTConfig, device=None, tp=None):
        super().__init__("gpt_embeddings")
        self.cfg, self.tp = cfg, _tp_on(tp)
        tpd = self.tp.world_size if self.tp else 1
        dt = _dt(cfg.dtype)
        self.word_embeddings = _param([cfg.vocab_size // tpd, cfg.hidden_size], device, dt, cfg.initializer_range)
        self.position_embeddings = _param([cfg.max_position_embeddings, cfg.hidden_size], device, dt,
                                          cfg.initializer_range)
        if self.tp:
            self.word_embeddings.is_distributed = True

    def forward(self, input_ids, position_ids=None):
        if self.tp:
            from ..distributed.fleet.mp_layers import vocab_parallel_embedding

            x = vocab_parallel_embedding(input_ids, self.word_embeddings, self.tp.group)
        else:
            x = ops.embedding(input_ids, self.word_embeddings)
        if position_ids is not None:
            return ops.add(x, ops.embedding(position_ids, self.position_embeddings))
        return ops.position_add(x, self.position_embeddings)


class GPTForCausalLM(Layer):
    def __init__(self, cfg: GPTConfig, device=None, tp=None):
        super().__init__("gpt")
        self.cfg, self.tp = cfg, _tp_on(tp)
        dt = _dt(cfg.dtype)
        self.embeddings = GPTEmbeddings(cfg, device, self.tp)
        self.layers = torch.nn.ModuleList([GPTDecoderLayer(cfg, device, i, self.tp)
                                           for i in range(cfg.num_hidden_layers)])
        self.ln_f_w = _param([cfg.hidden_size], device, dt, value=1.0)
        self.ln_f_b = _param([cfg.hidden_size], device, dt, value=0.0)
        self.ln_f_w.no_weight_decay = self.ln_f_b.no_weight_decay = True

    def hidden_states(self, input_ids):
        x = self.embeddings(input_ids)
        residual = None
        for layer in self.layers:
            if self.cfg.recompute and self.training and _tape.current() is not None:
                x, residual = _tape.checkpoint(layer, x, residual)  # recomputed on the framework tape
            elif self.cfg.recompute and self.training and torch.is_grad_enabled():
                x, residual = torch.utils.checkpoint.checkpoint(layer, x, residual, use_reentrant=False)
            else:
                x, residual = layer(x, residual)
        y, _ = ops.layer_norm(x, self.ln_f_w, self.ln_f_b, self.cfg.layer_norm_eps, residual=residual)
        return y

    def forward(self, input_ids, labels=None):
        y = self.hidden_states(input_ids)
        w = self.embeddings.word_embeddings  # tied LM head: logits = y @ E^T
        if self.tp:
            from ..distributed.fleet.mp_layers import parallel_cross_entropy

            logits = ops.linear_t(self.tp.copy_to_region(y), w)
            return logits if labels is None else parallel_cross_entropy(logits, labels, self.tp.group)
        logits = ops.linear_t(y, w)
        if labels is None:
            return logits
        return ops.softmax_cross_entropy(logits, labels, inplace_grad=True)


def gpt_flops_per_token(cfg: GPTConfig, seq_len: int) -> float:
    H, L, V, I = cfg.hidden_size, cfg.num_hidden_layers, cfg.vocab_size, cfg.ffn
    gemm = 2 * (3 * H * H + H * H + 2 * H * I)
    attn = 2 * 2 * seq_len * H / 2
    return 3 * (L * (gemm + attn) + 2 * H * V)


def shard_gpt_state_dict(full: dict, cfg: GPTConfig, rank: int, world: int) -> dict:
    """Full GPT state dict -> tensor-parallel shard (per-head split of the packed QKV)."""
    if world == 1:
        return dict(full)
    out = {}
    nh, D = cfg.num_attention_heads, cfg.head_dim
    for k, v in full.items():
        if k.endswith("qkv_w"):
            H = v.shape[0]
            out[k] = v.view(H, 3, nh, D).chunk(world, dim=2)[rank].reshape(H, -1).contiguous()
        elif k.endswith("qkv_b"):
            out[k] = v.view(3, nh, D).chunk(world, dim=1)[rank].reshape(-1).contiguous()
        elif k.endswith("fc1_w"):
            out[k] = v.chunk(world, dim=1)[rank].contiguous()
        elif k.endswith("fc1_b"):
            out[k] = v.chunk(world, dim=0)[rank].contiguous()
        elif k.endswith("out_w") or k.endswith("fc2_w") or k.endswith("word_embeddings"):
            out[k] = v.chunk(world, dim=0)[rank].contiguous()
        else:
            out[k] = v.clone()
    return out


# ------------------------------------------------------------------ pipeline
class GPTEmbeddingPipe(GPTEmbeddings):
    pass


class GPTDecoderLayerPipe(GPTDecoderLayer):
    pass


class GPTHeadPipe(Layer):
    """Final LayerNorm; the tied LM-head GEMM is applied by the shared embedding call."""

    def __init__(self, cfg: GPTConfig, device=None, tp=None):
        super().__init__("gpt_head")
        dt = _dt(cfg.dtype)
        self.cfg, self.tp = cfg, _tp_on(tp)
        self.ln_f_w = _param([cfg.hidden_size], device, dt, value=1.0)
        self.ln_f_b = _param([cfg.hidden_size], device, dt, value=0.0)

    def forward(self, x, residual):
        y, _ = ops.layer_norm(x, self.ln_f_w, self.ln_f_b, self.cfg.layer_norm_eps, residual=residual)
        return self.tp.copy_to_region(y) if self.tp else y


def _tied_head(emb, y):
    return ops.linear_t(y, emb.word_embeddings)


class GPTPretrainingCriterion:
    def __init__(self, tp=None):
        self.tp = _tp_on(tp)

    def __call__(self, logits, labels):
        if self.tp:
            from ..distributed.fleet.mp_layers import parallel_cross_entropy

            return parallel_cross_entropy(logits, labels, self.tp.group)
        return ops.softmax_cross_entropy(logits, labels, inplace_grad=True)


def gpt_pipeline_descs(cfg: GPTConfig, device=None, tp=None):
    from ..distributed.fleet.pipeline import LayerDesc, SharedLayerDesc

    descs = [SharedLayerDesc("embed", GPTEmbeddingPipe, None, "word_embeddings", cfg, device, tp)]
    descs += [LayerDesc(GPTDecoderLayerPipe, cfg, device, i, tp) for i in range(cfg.num_hidden_layers)]
    descs.append(LayerDesc(GPTHeadPipe, cfg, device, tp))
    descs.append(SharedLayerDesc("embed", GPTEmbeddingPipe, _tied_head, "word_embeddings", cfg, device, tp))
    return descs
