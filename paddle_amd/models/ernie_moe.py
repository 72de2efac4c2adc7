"""ERNIE-MoE: decoder-only LM with mixture-of-experts FFNs, expert parallelism over
an all-to-all group and optional fp8 expert weights (BASELINE.json config
"ERNIE-MoE Fleet expert-parallel all-to-all + fp8 MFMA weights").

Not in the reference (no MoE / all-to-all anywhere).  Architecture
follows the ERNIE-4.5-MoE family: pre-RMSNorm blocks with rotary attention (the
LLaMA attention path: fused QKV GEMM + fused rope/flash-attention kernel), the
first ``first_k_dense`` layers use a dense SwiGLU MLP, the rest an MoE FFN with
``num_experts`` SwiGLU experts, top-k softmax gating and a GShard auxiliary
load-balancing loss (``aux_loss_coeff``), optionally plus shared (always-on)
experts.  Expert GEMMs can run in fp8 (e4m3 weights, see :mod:`..ops.fp8`).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from .. import ops
from ..distributed.fleet.moe import MoELayer, TopKGate
from ..nn import Layer
from ..ops import grouped as _grouped
from ..ops.fp8 import fp8_linear
from ..ops.fused import param_ready
from .llama import _dt, _param


@dataclass
class ErnieMoEConfig:
    vocab_size: int = 103424
    hidden_size: int = 2560
    intermediate_size: int = 12288       # dense MLP
    moe_intermediate_size: int = 1536    # per expert
    num_hidden_layers: int = 28
    num_attention_heads: int = 20
    num_key_value_heads: int = 4
    num_experts: int = 64
    num_shared_experts: int = 0
    top_k: int = 6
    first_k_dense: int = 1
    capacity_factor: float | None = None
    aux_loss_coeff: float = 1e-2
    max_position_embeddings: int = 4096
    rms_norm_eps: float = 1e-5
    rope_theta: float = 500000.0
    initializer_range: float = 0.02
    use_fp8_experts: bool = False
    grouped_experts: bool = False         # ragged grouped GEMMs over all local experts (ops/grouped.py)
    dtype: str = "bfloat16"

    @property
    def head_dim(self):
        return self.hidden_size // self.num_attention_heads

    @property
    def kv_heads(self):
        return self.num_key_value_heads or self.num_attention_heads


ERNIE_MOE_CONFIGS = {
    # ERNIE-4.5-21B-A3B-like shape
    "ernie-moe-21b-a3b": dict(),
    # same block shapes, 8 layers: fits one MI355X with unsharded optimizer state
    "ernie-moe-a3b-8l": dict(num_hidden_layers=8),
    "ernie-moe-tiny": dict(vocab_size=512, hidden_size=128, intermediate_size=256, moe_intermediate_size=64,
                           num_hidden_layers=3, num_attention_heads=4, num_key_value_heads=2, num_experts=4,
                           top_k=2, max_position_embeddings=128),
}


class SwiGLUExpert(Layer):
    def __init__(self, H, I, device, dt, std, fp8=False):
        super().__init__("moe_expert")
        self.gate_up = _param([H, 2 * I], device, dt, std)
        self.down = _param([I, H], device, dt, std)
        self.fp8 = fp8

    def forward(self, x):
        lin = fp8_linear if self.fp8 else ops.linear
        return lin(ops.swiglu(lin(x, self.gate_up)), self.down)


class GroupedSwiGLUExperts(Layer):
    """All local experts of one MoE layer as stacked weights: gate_up [n, H, 2I],
    down [n, I, H].  On the GPU ``forward_grouped`` runs the expert-sorted tokens
    through :mod:`..ops.grouped` -- ragged grouped MFMA GEMMs (each workgroup reads
    its expert's row range, no padding) with the fused SwiGLU kernel between them
    and per-expert dW accumulated into the fp32 main_grad -- in place of ``n``
    separate GEMM chains, which are launch-bound at 64 experts x ~768 tokens
    (ernie-moe-a3b-8l ran at 12 % MFU that way).  The CPU path pads each expert to
    the largest count and uses batched matmuls.  Expert ``e`` is initialised from
    the same per-expert seed as ``SwiGLUExpert`` so the layout (grouped or not, any
    EP degree) does not change the model.  Reference: the MoE layer of Fleet
    (SURVEY.md §2.5 EP row) runs experts one by one."""

    def __init__(self, H, I, experts, device, dt, std, seed_of, fp8=False):
        super().__init__("moe_grouped_experts")
        self.fp8 = fp8
        gu, dn = [], []
        state = torch.random.get_rng_state()
        for e in experts:
            torch.manual_seed(seed_of(e))
            gu.append(_param([H, 2 * I], device, dt, std).data)
            dn.append(_param([I, H], device, dt, std).data)
        torch.random.set_rng_state(state)
        self.gate_up = torch.nn.Parameter(torch.stack(gu))
        self.down = torch.nn.Parameter(torch.stack(dn))
        self.num_experts = len(experts)

    def forward_grouped(self, x, counts):
        """``counts``: rows per local expert (device tensor: no host sync on the GPU
        path; or host ints)."""
        if x.shape[0] == 0:
            return x
        param_ready(self.gate_up)
        param_ready(self.down)
        if self.fp8 and _grouped.supported_f8(x, self.gate_up, self.down):
            return _grouped.grouped_swiglu_mlp(x, self.gate_up, self.down, counts, fp8=True)
        if _grouped.supported(x, self.gate_up, self.down):
            return _grouped.grouped_swiglu_mlp(x, self.gate_up, self.down, counts)
        if torch.is_tensor(counts):
            counts = counts.tolist()
        n, N = self.num_experts, x.shape[0]
        C = (max(counts) + 15) // 16 * 16
        ct = torch.tensor(counts, device=x.device)
        e_of_row = torch.repeat_interleave(torch.arange(n, device=x.device), ct, output_size=N)
        starts = torch.cumsum(ct, 0) - ct
        dest = e_of_row * C + (torch.arange(N, device=x.device) - starts[e_of_row])
        xp = x.new_zeros(n * C, x.shape[1]).index_copy(0, dest, x).view(n, C, -1)
        h = ops.swiglu(torch.bmm(xp, self.gate_up.to(x.dtype)))
        return torch.bmm(h, self.down.to(x.dtype)).view(n * C, -1).index_select(0, dest)


class ErnieMoEDecoderLayer(Layer):
    def __init__(self, cfg: ErnieMoEConfig, device=None, layer_idx=0, ep_group=None):
        super().__init__("ernie_moe_decoder")
        self.cfg = cfg
        H, D, dt, std = cfg.hidden_size, cfg.head_dim, _dt(cfg.dtype), cfg.initializer_range
        self.nh, self.nkv = cfg.num_attention_heads, cfg.kv_heads
        self.input_layernorm = _param([H], device, dt, value=1.0)
        self.qkv_proj = _param([H, (self.nh + 2 * self.nkv) * D], device, dt, std)
        self.o_proj = _param([self.nh * D, H], device, dt, std / math.sqrt(2 * cfg.num_hidden_layers))
        self.post_attention_layernorm = _param([H], device, dt, value=1.0)
        for n in ("input_layernorm", "post_attention_layernorm"):
            getattr(self, n).no_weight_decay = True
        self.is_moe = layer_idx >= cfg.first_k_dense
        if self.is_moe:
            from ..parallel import comm

            ep = comm.get_world_size(ep_group)
            if cfg.num_experts % ep:
                raise ValueError("num_experts must be divisible by the expert-parallel degree")
            r = comm.get_rank(ep_group)
            n_local = cfg.num_experts // ep
            experts = []
            if cfg.grouped_experts:
                experts = GroupedSwiGLUExperts(H, cfg.moe_intermediate_size, range(r * n_local, (r + 1) * n_local),
                                               device, dt, std, lambda e: 7919 * (layer_idx + 1) + e,
                                               fp8=cfg.use_fp8_experts)
            for e in (range(r * n_local, (r + 1) * n_local) if isinstance(experts, list) else ()):
                # per-expert seed: expert e has the same init whatever the EP layout
                state = torch.random.get_rng_state()
                torch.manual_seed(7919 * (layer_idx + 1) + e)
                experts.append(SwiGLUExpert(H, cfg.moe_intermediate_size, device, dt, std, cfg.use_fp8_experts))
                torch.random.set_rng_state(state)
            gate = TopKGate(H, cfg.num_experts, cfg.top_k, "gshard", cfg.capacity_factor)
            gate.to(device=device)
            self.moe = MoELayer(H, experts, gate=gate, group=ep_group, capacity_factor=cfg.capacity_factor)
            self.shared = SwiGLUExpert(H, cfg.moe_intermediate_size * cfg.num_shared_experts, device, dt, std) \
                if cfg.num_shared_experts else None
        else:
            self.mlp = SwiGLUExpert(H, cfg.intermediate_size, device, dt, std)

    def forward(self, x, residual, cos, sin):
        cfg, eps = self.cfg, self.cfg.rms_norm_eps
        if residual is None:
            h = x
            y = ops.rms_norm(x, self.input_layernorm, eps)
        else:
            y, h = ops.rms_norm(x, self.input_layernorm, eps, residual=residual)
        a = ops.linear(ops.rope_attention(ops.linear(y, self.qkv_proj), cos, sin, self.nh, self.nkv, causal=True),
                       self.o_proj)
        y2, h2 = ops.rms_norm(a, self.post_attention_layernorm, eps, residual=h)
        if self.is_moe:
            m = self.moe(y2)
            if self.shared is not None:
                m = m + self.shared(y2)
        else:
            m = self.mlp(y2)
        return m, h2


class ErnieMoEForCausalLM(Layer):
    def __init__(self, cfg: ErnieMoEConfig, device=None, ep_group=None):
        super().__init__("ernie_moe")
        self.cfg = cfg
        dt, std, H = _dt(cfg.dtype), cfg.initializer_range, cfg.hidden_size
        self.embed_tokens = _param([cfg.vocab_size, H], device, dt, std)
        self.layers = torch.nn.ModuleList([ErnieMoEDecoderLayer(cfg, device, i, ep_group)
                                           for i in range(cfg.num_hidden_layers)])
        self.norm = _param([H], device, dt, value=1.0)
        self.norm.no_weight_decay = True
        self.lm_head = _param([H, cfg.vocab_size], device, dt, std)
        cos, sin = ops.rope_tables(cfg.max_position_embeddings, cfg.head_dim, cfg.rope_theta, device=device)
        self.register_buffer("rope_cos", cos, persistent=False)
        self.register_buffer("rope_sin", sin, persistent=False)

    def forward(self, input_ids, labels=None):
        x = ops.embedding(input_ids, self.embed_tokens)
        residual = None
        aux = []
        for layer in self.layers:
            x, residual = layer(x, residual, self.rope_cos, self.rope_sin)
            if layer.is_moe and layer.moe.l_aux is not None:
                aux.append(layer.moe.l_aux)
        y, _ = ops.rms_norm(x, self.norm, self.cfg.rms_norm_eps, residual=residual)
        logits = ops.linear(y, self.lm_head)
        if labels is None:
            return logits
        loss = ops.softmax_cross_entropy(logits, labels, inplace_grad=True)
        self.last_ce = loss.detach()  # the next-token cross-entropy alone (loss adds the balance term)
        if aux and self.cfg.aux_loss_coeff:
            loss = ops.add(loss, ops.scale(ops.stack_mean(aux), self.cfg.aux_loss_coeff))
        return loss
