"""paddle_amd operator library: fused gfx950 HIP kernels with CPU reference paths."""
from . import fused, optim  # noqa: F401
from .fused import (apply_rotary, embedding, flash_attention, flash_attention_varlen, layer_norm, linear, linear_t,  # noqa: F401
                    linear_gelu, rms_norm, packed_attention, rope_attention, rope_tables, softmax, softmax_cross_entropy, swiglu,
                    deinterleave_gate_up, interleave_gate_up, qkv_rope_attention, swiglu_mlp, add, scale,
                    position_add, mean_valid, cross_entropy_tokens, reshape, stack_mean,
                    row_gather, concat_rows)
